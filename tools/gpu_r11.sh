#!/bin/bash
# GPU suite, the tolerance margin probe and the driver command per rtol
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r11}; mkdir -p "$OUT"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "=== $name rc=$rc" >&2; tail -n 3 "$OUT/$name.out" >&2
  if [ $rc -ne 0 ]; then echo "stop after $name" >&2; tail -n 20 "$OUT/$name.err" >&2; exit $rc; fi
}
[ -z "$SKIP_TESTS" ] && step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread ${PYTEST_ARGS}
[ -z "$SKIP_MARGIN" ] && step margin_100 400 python -u tools/margin_probe.py --start 100 --window 50 --rtols ${RTOLS:-1e-7,5e-8,3e-8}
for r in ${BENCH_RTOLS:-1e-7 5e-8}; do
  step bench_$r 300 python -u bench.py --no-cpu-baseline --no-secondary --warmup 5 --steps 20 --rtol-pres $r
done
