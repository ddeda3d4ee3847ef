#!/bin/bash
# k_sl under the locator knobs: default (lattice), PUCFEM_SL_PROBE=1 (no rank count), records locator.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-slv}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
B="--gpus 1 --steps 8 --warmup 3 --no-cpu-baseline --no-secondary --kernel-table"
for v in lattice probe records; do
  case $v in
    lattice) E="";; probe) E="PUCFEM_SL_PROBE=1";; records) E="PUCFEM_SL_RECORDS=1";;
  esac
  env $E timeout -k 10 300 python -u bench.py $B > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v failed" >&2; tail -5 "$OUT/$v.err" >&2; exit 1; }
  python -c "import json,sys;d=json.load(open('$OUT/$v.json'));k=d['kernels'];print('$v', d['value'], k['k_sl']['avg_launch_ms'], k.get('k_sl_slow (general locate + rank count)',{}).get('avg_launch_ms'))" >&2
done
