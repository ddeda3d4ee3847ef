#!/bin/bash
# bit comparison of the default library against libpucfem.$1.so (tools/bitcmp.py runs), then the driver A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=$1; shift
for args in "5 60" "7 30"; do
  timeout -k 10 300 python tools/bitcmp.py $args || exit 1
  PUCFEM_LIB_VARIANT=$V timeout -k 10 300 python tools/bitcmp.py $args || exit 1
done
PUCFEM_CGCG=1 timeout -k 10 300 python tools/bitcmp.py 4 40 || exit 1
PUCFEM_CGCG=1 PUCFEM_LIB_VARIANT=$V timeout -k 10 300 python tools/bitcmp.py 4 40 || exit 1
