cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r2p; mkdir -p $OUT
i=0
for a in "--proj-k 24" "--proj-k 16" "--proj-k 32" "--proj-k 12" "--proj-k 24 --rtol-pres 1e-7"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-kernel-timing --warmup 5 --steps 20 $a > $OUT/b$i.out 2> $OUT/b$i.err || exit 1
  python -c "
import json;r=json.load(open('$OUT/b$i.out'));it=r['cg_iters_per_step']
print('$a', round(r['value'],2), 'p', sum(it['p']), 'p2', sum(it['p2']))" >&2
  i=$((i+1))
done
