#!/bin/bash
# PMC passes on the semi-Lagrangian kernels of the bench step (one pass per counter group).
# Usage: tools/gpu_sl_pmc.sh TAG [kernel regex]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-slpmc}; RX=${2:-k_sl}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1)); rm -rf /tmp/slpmc_$i
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "$RX" -d /tmp/slpmc_$i -o run --output-format csv -- \
    python $ROOT/bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-kernel-timing > $OUT/pass$i.out 2>&1 || { echo "pass $i failed" >&2; tail -5 $OUT/pass$i.out >&2; exit 1; }
  find /tmp/slpmc_$i -name "*counter_collection.csv" -exec cp {} $OUT/pass$i.csv \;
done
ls -la $OUT >&2
