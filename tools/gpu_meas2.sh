#!/bin/bash
# The driver's bench command + a kernel trace of its timed window (tools/gpu_meas.sh, tests skipped), then a
# kernel trace of the mesh_fine step (tools/fine_probe.py: per-launch listing of the last graph replays)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${1:-meas}
SKIP_TESTS=1 bash tools/gpu_meas.sh "$TAG" || exit $?
OUT="$ROOT/gpurun_out/$TAG"
cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/fine_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/fine_$TAG -o run --output-format csv -- \
  python "$ROOT/tools/fine_probe.py" 200 > "$OUT/fine_probe.txt" 2> "$OUT/fine_probe.err"
rc=$?; echo "fine rc=$rc" >&2; cat "$OUT/fine_probe.txt" >&2; [ $rc -ne 0 ] && exit $rc
f=$(find /tmp/fine_$TAG -name "*kernel_trace.csv" | head -1)
python "$ROOT/tools/trace_replay.py" "$f" 3 > "$OUT/fine_replay_trace.txt"
find /tmp/fine_$TAG -name "*kernel_stats.csv" -exec cp {} "$OUT/fine_kernel_stats.csv" \;
tail -3 "$OUT/fine_replay_trace.txt" >&2
timeout -k 10 120 python "$ROOT/tools/fine_probe.py" 2000 >&2
cd "$ROOT"
PUCFEM_DEEP_REPORT=1 timeout -k 10 240 python -u tools/comm_probe.py 7 8 2 > "$OUT/comm_probe_report.txt" 2>&1
rc=$?; grep -E "\[deep\]|per pressure" "$OUT/comm_probe_report.txt" >&2; exit $rc
