#!/bin/bash
# A/B of the driver command (window + steady leg): k_sl grid caps, projection basis sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ab}; mkdir -p "$OUT"; shift
B="python -u bench.py --no-cpu-baseline --no-secondary --warmup 5 --steps 20"
run() { local name=$1; shift; echo "=== $name" >&2; timeout -k 10 200 env "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "fail $name" >&2; exit 1; };
  python -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value'],2), 'steady', round(d['steady']['steps_per_s'],2))" >&2; }
for rep in 1 2; do
run base_$rep $B
run slb1024_$rep PUCFEM_SL_BLOCKS=1024 $B
run slb2048_$rep PUCFEM_SL_BLOCKS=2048 $B
run pk16_$rep $B --proj-k 16
run pk12_$rep $B --proj-k 12
done
