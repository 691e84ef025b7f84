# Whole-bench A/B of the 2D stencil tile height (GPU box): bash tools/ab_st.sh
set -e
mkdir -p gpurun_out
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels'];j=[v['avg_us'] for n,v in k.items() if n.startswith('jv_fd')];print(d['value'], j)" "$1"; }
for r in 1 2; do
  for w in bratu2d heat2d; do
    NK_ST_BLOCKS=2048 NK_ST_MAXROWS=64 timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --prof-every 8 > gpurun_out/ab_st_old_$w.$r.log 2>&1; echo "$w old (2048 tiles, <= 64 rows) round $r $(val gpurun_out/ab_st_old_$w.$r.log)"
    timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --prof-every 8 > gpurun_out/ab_st_new_$w.$r.log 2>&1; echo "$w new (1024 tiles, <= 32 rows) round $r $(val gpurun_out/ab_st_new_$w.$r.log)"
  done
done
