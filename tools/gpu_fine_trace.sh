#!/bin/bash
# Kernel trace of the mesh_fine step (tools/fine_probe.py, per-launch listing of the last graph replays by
# tools/trace_replay.py); with TESTS=1 the whole -m gpu suite first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${1:-fine}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.out" 2> "$OUT/pytest_gpu.err"
  rc=$?; tail -3 "$OUT/pytest_gpu.out" >&2; [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/fine_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/fine_$TAG -o run --output-format csv -- \
  python "$ROOT/tools/fine_probe.py" 200 > "$OUT/fine_probe.txt" 2> "$OUT/fine_probe.err"
rc=$?; echo "fine rc=$rc" >&2; cat "$OUT/fine_probe.txt" >&2; [ $rc -ne 0 ] && exit $rc
f=$(find /tmp/fine_$TAG -name "*kernel_trace.csv" | head -1)
python "$ROOT/tools/trace_replay.py" "$f" 3 > "$OUT/fine_replay_trace.txt"
gzip -c "$f" > "$OUT/fine_kernel_trace.csv.gz"
find /tmp/fine_$TAG -name "*kernel_stats.csv" -exec cp {} "$OUT/fine_kernel_stats.csv" \;
tail -3 "$OUT/fine_replay_trace.txt" >&2
cd "$ROOT" && timeout -k 10 120 python tools/fine_probe.py 2000 >&2
