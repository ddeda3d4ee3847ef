#!/bin/bash
# the driver command twice (no secondary legs) + optional pytest filter; usage: gpu_quick_bench.sh TAG [pytest -k expr]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-quick}; mkdir -p "$OUT"
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "$2" > $OUT/pytest.txt 2>&1; rc=$?
  echo "pytest rc=$rc" >&2; tail -n 2 $OUT/pytest.txt >&2; [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary --warmup 5 --steps 20 > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/bench_$rep.json').read().strip().splitlines()[-1]); print('bench', round(d['value'],2), 'steady', round(d['steady']['steps_per_s'],2), 'launches', round(d['launches_per_step'],1), d['roofline']['kernel'], round(d['roofline']['frac'],3))" >&2
done
