#!/bin/bash
# tolerance margin at L7 (steps 100-149 and 1000-1019 from a common state) and the driver command per rtol
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-margin}; mkdir -p "$OUT"
timeout -k 10 400 python -u tools/margin_probe.py --start 100 --window 50 --rtols 1e-7,5e-8,3e-8,2e-8 > "$OUT/margin_100.txt" 2>&1 || exit $?
for r in 1e-7 5e-8 3e-8; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-secondary --warmup 5 --steps 20 --rtol-pres $r > "$OUT/bench_$r.json" 2> "$OUT/bench_$r.err" || exit $?
done
timeout -k 10 300 python -u tools/margin_probe.py --start 1000 --window 20 --rtols 1e-7,5e-8,3e-8 > "$OUT/margin_1000.txt" 2>&1 || exit $?
