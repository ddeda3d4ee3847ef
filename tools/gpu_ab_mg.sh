#!/bin/bash
# Multigrid parameter A/B on the driver command (bench args per variant).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-mgab}; shift; mkdir -p $OUT
i=0
for a in "$@"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-kernel-timing --warmup 5 --steps 20 $a > $OUT/b$i.out 2> $OUT/b$i.err || exit 1
  python -c "
import json;r=json.load(open('$OUT/b$i.out'));it=r['cg_iters_per_step']
print('[$a]', round(r['value'],2), 'p', sum(it['p']), 'p2', sum(it['p2']), 'visc', sum(it['visc_2rhs']))" >&2
  i=$((i+1))
done
