#!/bin/bash
# Kernel trace of a bench run (rocprofv3 --kernel-trace only), kept gzip'd under gpurun_out/TAG for
# offline analysis (tools/trace_window.py, tools/trace_overlap.py).  Usage: tools/gpu_trace_keep.sh TAG [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${1:-trace}; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/tr_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/tr_$TAG -o run --output-format csv -- \
  python "$ROOT/bench.py" --no-cpu-baseline --no-secondary "$@" > "$OUT/bench.out" 2> "$OUT/bench.err"
rc=$?; echo "rocprof rc=$rc" >&2; [ $rc -ne 0 ] && { tail -5 "$OUT/bench.err" >&2; exit $rc; }
f=$(find /tmp/tr_$TAG -name "*kernel_trace.csv" | head -1)
gzip -c "$f" > "$OUT/kernel_trace.csv.gz"
python "$ROOT/tools/trace_window.py" "$f" --warmup 5 --steps 20 --top 60 > "$OUT/step_window.txt" && head -30 "$OUT/step_window.txt" >&2
