set -e
mkdir -p gpurun_out
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d['value'], d['kernels']['jv_fd_dot']['avg_us'], d['kernels']['mgs_sweep']['avg_us'])" "$1"; }
for r in 1 2; do
  for nb in 512 1024 2048 4096; do NK_ST_BLOCKS=$nb timeout -k 10 200 python bench.py --no-cpu-baseline --prof-every 8 > gpurun_out/ab_st$nb.$r.log 2>&1; echo "NK_ST_BLOCKS=$nb round $r $(val gpurun_out/ab_st$nb.$r.log)"; done
done
