#!/bin/bash
# alternating A/B of the driver command (no secondary legs): the default library vs each libpucfem.$VAR.so
# usage: gpu_ab_variants.sh TAG REPS VAR...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ab}; REPS=${2:-2}; shift 2; mkdir -p "$OUT"
B="python -u bench.py --no-cpu-baseline --no-secondary --warmup 5 --steps 20"
run() { local name=$1; shift; timeout -k 10 200 env "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "fail $name" >&2; tail -5 "$OUT/$name.err" >&2; exit 1; };
  python -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$name', round(d['value'],2), 'steady', round(d['steady']['steps_per_s'],2), {n.split()[0]: round(v['avg_launch_ms']*1e3,1) for n, v in k.items() if n.split()[0] in ('k_div','k_grad_proj','k_mdot2','k_pcomb','k_sl','k_vcheb_pair')})" >&2; }
for rep in $(seq 1 $REPS); do
  run base_$rep $B
  for v in "$@"; do run ${v}_$rep PUCFEM_LIB_VARIANT=$v $B; done
done
