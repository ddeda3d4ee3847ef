#!/bin/bash
# One measurement round on the GPU box:
#   parity tests -> bench line -> rocprofv3 kernel stats of the same command ->
#   two PMC passes (FETCH_SIZE, WRITE_SIZE; separate passes, kernel trace only) -> per-kernel HBM bytes.
# Usage: tools/gpu_round.sh TAG [bench args...]   (traces stay in /tmp; only summaries land in gpurun_out/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${1:-run}; shift
BARGS="$*"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "=== $name rc=$rc" >&2; tail -n 4 "$OUT/$name.out" >&2; tail -n 4 "$OUT/$name.err" >&2
  if [ $rc -ne 0 ]; then echo "stop after $name" >&2; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then step pytest_gpu 900 python -m pytest tests -m gpu -x -q; fi
step bench 900 python bench.py $BARGS
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_$TAG
step rocprof_stats 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG/stats -o run --output-format csv -- \
  python "$ROOT/bench.py" $BARGS
find /tmp/prof_$TAG/stats -name "*stats*.csv" -exec cp {} "$OUT/" \;
# per-kernel time over the bench's timed window (the driver schedule: --warmup W --steps K in BARGS)
TR=$(find /tmp/prof_$TAG/stats -name "*kernel_trace.csv" | head -1)
W=$(echo " $BARGS" | sed -n 's/.* --warmup \([0-9]*\).*/\1/p'); K=$(echo " $BARGS" | sed -n 's/.* --steps \([0-9]*\).*/\1/p')
[ -n "$TR" ] && python "$ROOT/tools/trace_window.py" "$TR" --warmup ${W:-20} --steps ${K:-20} --top 80 > "$OUT/step_window.txt"
if [ -z "$SKIP_PMC" ]; then
  step pmc_fetch 900 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d /tmp/prof_$TAG/fetch -o run --output-format csv -- \
    python "$ROOT/bench.py" $BARGS --steps 1 --warmup 1 --no-cpu-baseline --no-secondary
  step pmc_write 900 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d /tmp/prof_$TAG/write -o run --output-format csv -- \
    python "$ROOT/bench.py" $BARGS --steps 1 --warmup 1 --no-cpu-baseline --no-secondary
  cd "$ROOT"
  step pmc_parse 300 python tools/pmc_traffic.py /tmp/prof_$TAG/fetch /tmp/prof_$TAG/write "$OUT/pmc_traffic.json"
fi
ls -la "$OUT" >&2
