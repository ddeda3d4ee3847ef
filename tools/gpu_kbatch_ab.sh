#!/bin/bash
# isolated kernel_batch times of the default library vs variants: usage gpu_kbatch_ab.sh TAG KEY VAR...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-kb}; KEY=$2; shift 2; mkdir -p "$OUT"
B="python -u bench.py --no-cpu-baseline --no-secondary --warmup 3 --steps 5 --steady-after 0"
for v in base "$@"; do
  if [ "$v" = base ]; then E=""; else E="PUCFEM_LIB_VARIANT=$v"; fi
  timeout -k 10 200 env $E $B > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "fail $v" >&2; tail -5 "$OUT/$v.err" >&2; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1]); kb=d['kernel_batch']; print('$v', {k: (round(x['ms_batch']*1e3,1), round(x['GBps_batch'])) for k, x in kb.items() if '$KEY' in k})" >&2
done
