#!/bin/bash
# L7 bench line (driver command, no CPU legs) once per environment setting given as a quoted
# argument ("" = defaults), e.g. tools/gpu_env_ab.sh TAG "" "PUCFEM_MG_POST_COARSE=1"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-envab}; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
BARGS=${BARGS:---warmup 5 --steps 20}
i=0
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary $BARGS > "$OUT/bench$i.out" 2> "$OUT/bench$i.err"
  rc=$?; echo "[$e] rc=$rc" >&2
  [ $rc -ne 0 ] && { tail -3 "$OUT/bench$i.err" >&2; exit $rc; }
  python - "$OUT/bench$i.out" <<'PY' >&2
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
it = r['cg_iters_per_step']
print(f"  value {r['value']:.3f} steps/s  ms/step {r['ms_per_step']:.2f}  p {sum(it['p'])} p2 {sum(it['p2'])} visc {sum(it.get('visc_cheb_steps', it.get('visc_2rhs', [])))}")
for k, v in r.get("kernels", {}).items():
    print(f"    {k:40s} {v['avg_launch_ms']*1e3:8.1f} us")
PY
  i=$((i+1))
done
