#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r11h}; mkdir -p "$OUT"
B="python -u bench.py --no-cpu-baseline --no-secondary --warmup 5 --steps 20"
run() { local name=$1; shift; echo "=== $name" >&2; timeout -k 10 200 env "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "fail $name" >&2; exit 1; };
  python -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value'],2), 'steady', round(d['steady']['steps_per_s'],2), d['projection'], d['steady']['projection'], d['steady']['cg_iters_per_step'])" >&2; }
run base $B
run pk12 $B --proj-k 12
run pk16 $B --proj-k 16
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1; echo "pytest rc=$?" >&2; tail -n 3 $OUT/pytest_gpu.txt >&2
