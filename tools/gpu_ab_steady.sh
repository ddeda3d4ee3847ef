#!/bin/bash
# A/B of bench variants on one box: the driver window (5 + 20 steps) and the steady-state leg (steps
# 100-119) per variant.  Each argument is one variant: "ENV=v ... -- bench args" (either part optional).
# Usage: tools/gpu_ab_steady.sh TAG "" "-- --proj-k 16" "PUCFEM_PROJ_KEEP=8 -- --proj-k 24" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for v in "$@"; do
  envs=""; args="$v"
  case "$v" in *--*) envs="${v%%--*}"; args="${v#*--}";; esac
  case "$v" in *=*) [ "$envs" = "" ] && envs="$v" && args="";; esac
  kt="--no-kernel-timing"; [ -n "$KT" ] && kt=""  # KT=1: per-launch kernel events (the kernel table below)
  timeout -k 10 400 env $envs python bench.py --no-cpu-baseline --no-secondary $kt --warmup 5 --steps 20 \
    $args > "$OUT/b$i.out" 2> "$OUT/b$i.err"
  rc=$?
  python - "$OUT/b$i.out" "$v" <<'PY' >&2
import json, sys
try:
    r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
except Exception as e:
    print(f"[{sys.argv[2]}] no result: {e}"); sys.exit(0)
it = r["cg_iters_per_step"]; st = r.get("steady") or {}
si = st.get("cg_iters_per_step", {})
print(f"[{sys.argv[2]}] window {r['value']:.2f} steps/s ({r['launches_per_step']:.0f} launches/step, p+p2 "
      f"{sum(it['p']) + sum(it['p2'])}) | steady {st.get('steps_per_s', 0):.2f} steps/s "
      f"({st.get('launches_per_step', 0):.0f} launches/step, p+p2 {sum(si.get('p', [])) + sum(si.get('p2', []))})")
for k, v in sorted(r.get("kernels", {}).items(), key=lambda kv: -kv[1]["ms_per_step"])[:10]:
    print(f"    {k[:44]:44s} {v['ms_per_step']:.3f} ms/step  {v['avg_launch_ms'] * 1e3:7.1f} us  {v['achieved_GBps']:6.0f} GB/s")
PY
  [ $rc -ne 0 ] && { echo "variant [$v] rc=$rc" >&2; tail -3 "$OUT/b$i.err" >&2; exit $rc; }
  i=$((i+1))
done
exit 0
