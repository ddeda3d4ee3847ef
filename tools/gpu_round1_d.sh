#!/bin/bash
# parity tests (incl. multigrid) -> bench L7 (MG) -> rocprofv3 stats (trace kept in /tmp, only summaries copied)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" >&2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "=== $name rc=$rc" >&2; tail -n 12 "gpurun_out/$name.out" >&2; tail -n 6 "gpurun_out/$name.err" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name" >&2; exit $rc; fi
}
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step bench_l7 900 python bench.py
cd /tmp && export TMPDIR=/tmp
echo "=== rocprof" >&2
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_l7d -o run --output-format csv -- \
  python "$ROOT/bench.py" > "$ROOT/gpurun_out/prof_l7d.out" 2> "$ROOT/gpurun_out/prof_l7d.err"
rc=$?; echo "rocprof rc=$rc" >&2; tail -3 "$ROOT/gpurun_out/prof_l7d.err" >&2
mkdir -p "$ROOT/gpurun_out/prof_l7d"
find /tmp/prof_l7d -name "*stats*.csv" -exec cp {} "$ROOT/gpurun_out/prof_l7d/" \;
ls -la "$ROOT/gpurun_out/prof_l7d" >&2
exit $rc
