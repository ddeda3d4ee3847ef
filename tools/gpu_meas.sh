#!/bin/bash
# The driver's bench command (all legs: cpu_baseline, L5, mesh_fine) and a kernel trace of its timed
# window (tools/trace_window.py).  Usage: tools/gpu_meas.sh TAG [extra bench args]
#   SKIP_TESTS unset: the GPU parity suite first.  SKIP_TRACE set: no trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${1:-meas}; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.out" 2>&1
  rc=$?; echo "pytest rc=$rc" >&2; grep -E "passed|failed|Error|error" "$OUT/pytest_gpu.out" | tail -15 >&2
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 900 python bench.py --warmup 5 --steps 20 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc" >&2; tail -3 "$OUT/bench.err" >&2; cat "$OUT/bench.json" >&2
[ $rc -ne 0 ] && exit $rc
[ -n "$SKIP_TRACE" ] && exit 0
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/tr_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/tr_$TAG -o run --output-format csv -- \
  python "$ROOT/bench.py" --warmup 5 --steps 20 --no-cpu-baseline --no-secondary "$@" > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
rc=$?; echo "rocprof rc=$rc" >&2; [ $rc -ne 0 ] && { tail -5 "$OUT/trace_bench.err" >&2; exit $rc; }
f=$(find /tmp/tr_$TAG -name "*kernel_trace.csv" | head -1)
find /tmp/tr_$TAG -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python "$ROOT/tools/trace_window.py" "$f" --warmup 5 --steps 20 --top 60 > "$OUT/step_window.txt"
rc=$?; head -40 "$OUT/step_window.txt" >&2
exit $rc
