#!/bin/bash
# Per-launch event timing against rocprof and against untimed steps (L7, one GPU):
#   A: default bench (events on the finest-level launches of the timed steps)
#   B: the same without the projection side stream
#   C: steps without kernel events (step time only)
#   D: rocprofv3 --stats of a run whose kernels are nearly all timed-region launches (1 warm-up step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT="$ROOT/gpurun_out/${1:-tab}"; mkdir -p "$OUT"
Q="--no-cpu-baseline --no-secondary"
run() { local n=$1; shift; echo "=== $n" >&2; timeout -k 10 600 "$@" > "$OUT/$n.out" 2> "$OUT/$n.err" || { echo "stop after $n" >&2; tail -5 "$OUT/$n.err" >&2; exit 1; }; }
run A python bench.py $Q
PUCFEM_NO_SIDE_STREAM=1 run B python bench.py $Q
run C python bench.py $Q --no-kernel-timing
cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/prof_tab
run D rocprofv3 --kernel-trace --stats -d /tmp/prof_tab -o run --output-format csv -- python "$ROOT/bench.py" $Q --warmup 1
find /tmp/prof_tab -name "*stats*.csv" -exec cp {} "$OUT/" \;
