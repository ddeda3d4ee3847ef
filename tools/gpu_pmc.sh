#!/bin/bash
# PMC traffic only (two passes: FETCH_SIZE, WRITE_SIZE; kernel trace only), parsed per kernel.
# Usage: tools/gpu_pmc.sh TAG [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-pmc}; shift
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/prof_$TAG
for c in FETCH_SIZE WRITE_SIZE; do
  d=/tmp/prof_$TAG/$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $c -d $d -o run --output-format csv -- \
    python "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-secondary "$@" > "$OUT/pmc_$c.out" 2> "$OUT/pmc_$c.err" \
    || { echo "pmc $c failed" >&2; tail -5 "$OUT/pmc_$c.err" >&2; exit 1; }
done
cp "$OUT/pmc_FETCH_SIZE.out" "$OUT/pmc_bench.out"  # (not bench.out: gpu_check_head.sh keeps the driver line there)
cd "$ROOT" && timeout -k 10 300 python tools/pmc_traffic.py /tmp/prof_$TAG/fetch /tmp/prof_$TAG/write "$OUT/pmc_traffic.json"
