#!/bin/bash
# k_sl_wave A/B on one box: SL tests, the driver command with and without the wave pass, a window trace, mesh_fine
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-absl}; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_parity.py -k "semilagrange" > "$OUT/pytest_sl.txt" 2>&1
rc=$?; tail -2 "$OUT/pytest_sl.txt" >&2; [ $rc -ne 0 ] && exit $rc
B="--warmup 5 --steps 20 --no-cpu-baseline --no-secondary"
for v in 1 0 1; do
  PUCFEM_SL_WAVE=$v timeout -k 10 300 python bench.py $B > "$OUT/bench_w$v.json" 2> "$OUT/bench_w$v.err" || exit 1
  python -c "import json,sys; d=json.loads(open('$OUT/bench_w$v.json').read().strip().splitlines()[-1]); print('SL_WAVE=$v', round(d['value'],2), 'steady', round(d['steady']['steps_per_s'],1))" >&2
done
cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/tr_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/tr_$TAG -o run --output-format csv -- \
  python "$ROOT/bench.py" $B > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || exit 1
f=$(find /tmp/tr_$TAG -name "*kernel_trace.csv" | head -1)
python "$ROOT/tools/trace_window.py" "$f" --warmup 5 --steps 20 --top 40 > "$OUT/step_window.txt"
head -3 "$OUT/step_window.txt" >&2; grep -E "k_sl" "$OUT/step_window.txt" >&2
cd "$ROOT" && timeout -k 10 120 python tools/fine_probe.py 2000 >&2
