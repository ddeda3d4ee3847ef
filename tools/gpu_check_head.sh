#!/bin/bash
# Parity at HEAD on the GPU box: the full `-m gpu` suite (verbose, per-test time limit), smoke(),
# then the driver's bench command. Every step has its own time limit; the script stops at the
# first failure. Usage: tools/gpu_check_head.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-head}
OUT="gpurun_out/$TAG"
mkdir -p "$OUT"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "=== $name rc=$rc" >&2; tail -n 6 "$OUT/$name.out" >&2; tail -n 4 "$OUT/$name.err" >&2
  if [ $rc -ne 0 ]; then echo "stop after $name" >&2; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread ${PYTEST_ARGS}
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [ -z "$SKIP_BENCH" ]; then step bench 600 python -u bench.py --gpus 1 --steps 20 --warmup 5; fi
if [ -n "$PROF" ]; then
  ROOT=$(pwd)
  rm -rf /tmp/prof_$TAG
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG/stats -o run \
     --output-format csv -- python "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
     --steady-after 0 > "$ROOT/$OUT/rocprof.out" 2> "$ROOT/$OUT/rocprof.err")
  rc=$?; echo "=== rocprof rc=$rc" >&2; tail -n 3 "$OUT/rocprof.err" >&2
  [ $rc -ne 0 ] && exit $rc
  find /tmp/prof_$TAG/stats -name "*stats*.csv" -exec cp {} "$OUT/" \;
  TR=$(find /tmp/prof_$TAG/stats -name "*kernel_trace.csv" | head -1)
  [ -n "$TR" ] && python tools/trace_window.py "$TR" --warmup 5 --steps 20 --top 90 > "$OUT/step_window.txt"
  # the roofline kernel over the launches the bench's events time (the last 5 timed steps), against the
  # profiled run's own bench line (rocprof.out)
  RK=$(python -c "import json,sys; print(json.loads(open('$OUT/rocprof.out').read().strip().splitlines()[-1])['roofline']['kernel'])")
  [ -n "$TR" ] && python tools/trace_window.py "$TR" --warmup 5 --steps 20 --last 5 --kernel "$RK" --top 30 > "$OUT/step_window_last5.txt"
  [ -n "$TR" ] && gzip -c "$TR" > "$OUT/kernel_trace.csv.gz"
fi
