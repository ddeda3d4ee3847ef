#!/bin/bash
# Kernel timeline of the bench's timed steps (rocprofv3 --kernel-trace only), summarised by
# tools/trace_step.py.  Usage: tools/gpu_trace.sh TAG [bench args]
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
python "$ROOT/tools/trace_step.py" "$f" ${LAST_MS:+--last-ms $LAST_MS} > "$OUT/trace_summary.txt" && cat "$OUT/trace_summary.txt" >&2
for p in "k_cheb<float, float, float, float, true, 1>" "k_cheb<float, float, double, float, true, 1>" \
         "k_resid<float, float, float, true, 1>" "k_cg_dir<1" "k_reduce" "k_bc_apply" "k_cg_upd<1>"; do
  python "$ROOT/tools/trace_launch.py" "$f" "$p" ${LAST_MS:+--last-ms $LAST_MS} >> "$OUT/trace_launch.txt"
done
cat "$OUT/trace_launch.txt" >&2
