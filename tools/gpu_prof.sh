#!/bin/bash
# Profile the driver's bench command: kernel-class table from the bench itself, then rocprofv3
# kernel-trace stats of the same command (summaries only into gpurun_out/TAG).
# Usage: tools/gpu_prof.sh TAG [extra bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-prof}; shift
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
BARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary $*"
timeout -k 10 600 python -u bench.py $BARGS --kernel-table > "$OUT/bench_table.json" 2> "$OUT/bench_table.err" || { echo "bench failed" >&2; tail -20 "$OUT/bench_table.err" >&2; exit 1; }
cut -c1-300 "$OUT/bench_table.json" >&2
cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run --output-format csv -- \
  python "$ROOT/bench.py" $BARGS > "$OUT/rocprof.out" 2> "$OUT/rocprof.err" || { echo "rocprof failed" >&2; tail -20 "$OUT/rocprof.err" >&2; exit 1; }
find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
find /tmp/prof_$TAG -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace.csv" \;
ls -la "$OUT" >&2
head -25 "$OUT/kernel_stats.csv" | cut -d, -f1-4 | cut -c1-200 >&2
