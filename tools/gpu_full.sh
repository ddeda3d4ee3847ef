#!/bin/bash
# the whole GPU suite, smoke(), then the driver command twice (no secondary legs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-full}; mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc" >&2; tail -n 2 $OUT/pytest_gpu.txt >&2; [ $rc -ne 0 ] && { grep -B5 -A30 "^_____" $OUT/pytest_gpu.txt | head -80 >&2; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo smoke failed >&2; tail -20 $OUT/smoke.txt >&2; exit 1; }
tail -n 2 $OUT/smoke.txt >&2
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary --warmup 5 --steps 20 > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/bench_$rep.json').read().strip().splitlines()[-1]); k=d['kernels']; print('bench', round(d['value'],2), 'steady', round(d['steady']['steps_per_s'],2), 'launches', round(d['launches_per_step'],1), d['roofline']['kernel'], round(d['roofline']['frac'],3), {n.split()[0]: round(v['avg_launch_ms']*1e3,1) for n, v in k.items()})" >&2
done
