# Resident-sweep hand-off: one polling wave (NK_RES_POLL1=1) vs four staggered ones (=2), per pass
# (tools/kbench_res.py, full residency and half) and whole bench, alternating (GPU box)
set -e
mkdir -p gpurun_out
for r in 1 2 3; do
  for p in 1 2; do
    echo "NK_RES_POLL1=$p round $r"
    NK_RES_POLL1=$p timeout -k 10 120 python tools/kbench_res.py --ks 30 --rvs 1000 --reps 3
    NK_RES_POLL1=$p timeout -k 10 120 python tools/kbench_res.py --n 33554432 --ks 30 --rvs 1006 --reps 2
  done
done
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d['value'], round(d['kernels']['mgs_sweep']['avg_us'],1))" "$1"; }
for r in 1 2; do
  for p in 1 2; do
    NK_RES_POLL1=$p timeout -k 10 200 python bench.py --no-cpu-baseline --prof-every 8 > gpurun_out/ab_poll.$p.$r.log 2>&1
    echo "bench NK_RES_POLL1=$p round $r $(val gpurun_out/ab_poll.$p.$r.log)"
  done
done
