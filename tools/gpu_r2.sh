#!/bin/bash
# Round-2 GPU check: the GPU test-suite (verbose, per-test time limit), then the driver's bench command.
# Usage: tools/gpu_r2.sh TAG [pytest -k expression]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r2}; K=${2:-}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${KA[@]}" \
  > "$OUT/pytest.out" 2> "$OUT/pytest.err"
rc=$?; echo "pytest rc=$rc" >&2; tail -30 "$OUT/pytest.out" >&2
[ $rc -ne 0 ] && exit $rc
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc" >&2; tail -3 "$OUT/bench.err" >&2; cut -c1-600 "$OUT/bench.json" >&2
fi
exit $rc
