#!/bin/bash
# Cold-cache face-stencil lab, then a kernel trace of the driver's bench command summarised over the
# timed window (tools/trace_window.py).  Usage: tools/gpu_lab_trace.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${1:-lab}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
if [ -x tools/_bin/cold_lab ]; then
  timeout -k 10 120 tools/_bin/cold_lab > "$OUT/cold_lab.txt" 2>&1; rc=$?
  cat "$OUT/cold_lab.txt" >&2; [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/tr_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/tr_$TAG -o run --output-format csv -- \
  python "$ROOT/bench.py" --no-cpu-baseline --no-secondary --no-kernel-timing --steps 20 --warmup 5 > "$OUT/bench.out" 2> "$OUT/bench.err"
rc=$?; echo "rocprof rc=$rc" >&2; [ $rc -ne 0 ] && { tail -5 "$OUT/bench.err" >&2; exit $rc; }
f=$(find /tmp/tr_$TAG -name "*kernel_trace.csv" | head -1)
python "$ROOT/tools/trace_window.py" "$f" --warmup 5 --steps 20 --top 70 > "$OUT/step_window.txt"
rc=$?; head -45 "$OUT/step_window.txt" >&2; exit $rc
