cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r10i
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --warmup 5 --steps 20 --steady-after 0 > gpurun_out/r10i/kt$i.out 2>/dev/null || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --warmup 5 --steps 20 --steady-after 0 --no-kernel-timing > gpurun_out/r10i/nokt$i.out 2>/dev/null || exit 1
done
python - <<'PY'
import json
for n in ("kt1","nokt1","kt2","nokt2"):
    r=json.loads(open(f"gpurun_out/r10i/{n}.out").read().strip().splitlines()[-1])
    print(n, round(r["value"],2))
PY
