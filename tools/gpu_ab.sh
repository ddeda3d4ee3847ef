#!/bin/bash
# GPU parity suite, then the L7 bench line for each variant given as a quoted argument list.
# Usage: tools/gpu_ab.sh TAG "" "--mg-f32-vals" "--index32" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.out" 2>&1
  rc=$?; echo "pytest rc=$rc" >&2; grep -E "passed|failed|Error|error" "$OUT/pytest_gpu.out" | tail -15 >&2
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for args in "$@"; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --no-secondary $args > "$OUT/bench$i.out" 2> "$OUT/bench$i.err"
  rc=$?; echo "bench[$args] rc=$rc" >&2; tail -2 "$OUT/bench$i.err" >&2
  python - "$OUT/bench$i.out" <<'PY' >&2
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"  value {r['value']:.3f} steps/s  ms/step {r['ms_per_step']:.2f}  iters {r['cg_iters_per_step']}  storage {r.get('storage')}")
for k, v in r["kernels"].items():
    print(f"  {k:40s} {v['avg_launch_ms']*1e3:8.1f} us  {v['achieved_GBps']:7.0f} GB/s  {v['bytes_per_launch']/1e6:8.1f} MB")
PY
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
