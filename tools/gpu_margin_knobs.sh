#!/bin/bash
# The L7 per-step margin test (steps 100-149 and 1000-1019 from a common state) under knob settings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-margin_knobs}; mkdir -p "$OUT"; shift
i=0
for e in "$@"; do
  echo "== $e" >&2
  env $e timeout -k 10 600 python -u -m pytest -x -q -s --timeout 550 --timeout-method thread \
    tests/test_gpu_scale_parity.py -k "per_step_past_transient" > "$OUT/m$i.out" 2>&1
  rc=$?; grep -E "common state" "$OUT/m$i.out" >&2; [ $rc -ne 0 ] && { tail -5 "$OUT/m$i.out" >&2; exit $rc; }
  i=$((i+1))
done
