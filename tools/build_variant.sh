#!/bin/bash
# A/B build of the library with extra compile definitions: libpucfem.NAME.so next to libpucfem.so,
# loaded when PUCFEM_LIB_VARIANT=NAME.  Usage: tools/build_variant.sh NAME -DPUCFEM_DIV_K=1 ...
set -e
cd "$(dirname "$0")/../puc-fluidsimulation-project_amd"
NAME=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -ffp-contract=off -Wall -Wno-unused-function \
  -I../include "$@" -o libpucfem.$NAME.so.tmp csrc/pucfem_api.hip csrc/pucfem_host.cpp -lrccl
mv libpucfem.$NAME.so.tmp libpucfem.$NAME.so
echo "built libpucfem.$NAME.so ($*)"
