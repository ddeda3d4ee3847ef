#!/bin/bash
# face_lab timings, then FETCH_SIZE / WRITE_SIZE per kernel (separate passes, kernel trace only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/lab; mkdir -p $OUT
timeout -k 10 120 tools/_bin/face_lab > $OUT/lab.txt 2>&1 || exit 1
cat $OUT/lab.txt >&2
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/lab_$c
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d /tmp/lab_$c -o run --output-format csv -- $ROOT/tools/_bin/face_lab > $OUT/pmc_$c.out 2>&1 || exit 1
  find /tmp/lab_$c -name "*counter_collection.csv" -exec cp {} $OUT/pmc_$c.csv \;
done
ls -la $OUT >&2
