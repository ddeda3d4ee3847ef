#!/bin/bash
# Can RCCL run 2 ranks on the single GPU of this box?  If so, check the multi-rank path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PUCFEM_DEVICE=0 NCCL_DEBUG=WARN
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 tools/dist_check.py 3 3 mg > gpurun_out/dist2.out 2> gpurun_out/dist2.err
rc=$?; echo "dist2 rc=$rc" >&2; tail -20 gpurun_out/dist2.out >&2; tail -25 gpurun_out/dist2.err >&2
exit $rc
