#!/bin/bash
# bench.py's kernel_batch table (kernels launched back to back outside the step) once per environment
# setting given as a quoted argument ("" = defaults; PUCFEM_LIB_VARIANT=NAME loads a tools/build_variant.sh
# build).  Usage: tools/gpu_kbatch.sh TAG "" "PUCFEM_LIB_VARIANT=divk1"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-kbatch}; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
BARGS=${BARGS:---warmup 5 --steps 20 --steady-after 0}
i=0
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary $BARGS > "$OUT/bench$i.out" 2> "$OUT/bench$i.err"
  rc=$?; echo "[$e] rc=$rc" >&2
  [ $rc -ne 0 ] && { tail -3 "$OUT/bench$i.err" >&2; exit $rc; }
  python - "$OUT/bench$i.out" <<'PY' >&2
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"  value {r['value']:.3f} steps/s")
for k, v in r.get("kernel_batch", {}).items():
    print(f"    {k:40s} batch {v['ms_batch']*1e3:8.1f} us  each {v['ms_each_event']*1e3:8.1f} us  {v['GBps_batch']:7.0f} GB/s")
PY
  i=$((i+1))
done
