#!/bin/bash
# L7 bench line + rocprofv3 kernel-trace stats of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 900 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_l7.json 2> gpurun_out/bench_l7.err
rc=$?; echo "bench rc=$rc" >&2; tail -5 gpurun_out/bench_l7.err >&2; cat gpurun_out/bench_l7.json >&2
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_l7" -o run --output-format csv -- \
  python "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > "$ROOT/gpurun_out/prof_l7.out" 2> "$ROOT/gpurun_out/prof_l7.err"
rc=$?; echo "rocprof rc=$rc" >&2; tail -3 "$ROOT/gpurun_out/prof_l7.err" >&2
find "$ROOT/gpurun_out/prof_l7" -name "*stats*" >&2
exit $rc
