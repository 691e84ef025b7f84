# Whole-bench A/B of the 3D F0 recomputation (k_st3l F0R, one wave less per SIMD): bash tools/ab_f0r3.sh
set -e
mkdir -p gpurun_out
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels'];j={n:round(v['avg_us'],1) for n,v in k.items() if n.startswith('jv_fd')};print(d['value'], j)" "$1"; }
for r in 1 2; do
  for w in "heat3d" "heat3d --global-n 512 --slab-of 8"; do
    t=$(echo $w | tr -d ' -')
    for f in 3 1; do
      NK_F0R=$f timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/ab_f0r3_${t}_$f.$r.log 2>&1
      echo "$w NK_F0R=$f round $r $(val gpurun_out/ab_f0r3_${t}_$f.$r.log)"
    done
  done
done
