#!/bin/bash
# First GPU validation: smoke -> GPU parity tests -> short bench probe.
# Each GPU step has its own time limit; stop at the first crash/timeout (rc not in {0,1}).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -n 30 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 900 python -m pytest tests -m gpu -x -q
run bench_l5 600 python bench.py --level 5 --steps 2 --warmup 1 --no-cpu-baseline
