#!/bin/bash
# A/B of bench.py argument sets on one box: the driver's schedule (--warmup 5 --steps 20), no CPU legs,
# no per-launch events.  Usage: tools/gpu_ab_args.sh TAG "args A" "args B" ...   (each run twice, interleaved)
# Words of the form PUCFEM_NAME=value in an argument set are environment settings for that run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  i=0
  for args in "$@"; do
    i=$((i + 1))
    envs=""; bargs=""
    for w in $args; do case "$w" in PUCFEM_*=*) envs="$envs $w";; *) bargs="$bargs $w";; esac; done
    env $envs timeout -k 10 300 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-secondary --no-kernel-timing $bargs \
      > "$OUT/ab_${i}_${rep}.json" 2> "$OUT/ab_${i}_${rep}.err" || { echo "run $i/$rep failed" >&2; tail -5 "$OUT/ab_${i}_${rep}.err" >&2; exit 1; }
    python -c "import json,sys; r=json.load(open('$OUT/ab_${i}_${rep}.json')); print('[$args] rep $rep: %.1f steps/s, %.0f launches/step, p-iters %s' % (r['value'], r['launches_per_step'], sum(r['cg_iters_per_step']['p'])+sum(r['cg_iters_per_step']['p2'])))" | tee -a "$OUT/summary.txt" >&2
  done
done
