# Whole-bench A/B of the 2D F0 recomputation per heat scheme: bash tools/ab_f0r2.sh
set -e
mkdir -p gpurun_out
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels'];j={n:round(v['avg_us'],1) for n,v in k.items() if n.startswith('jv_fd')};print(d['value'], j)" "$1"; }
for r in 1 2; do
  for w in "heat2d --scheme midpoint" "heat2d --scheme trapezoid" "heat2d --scheme trapezoid --bc periodic" "heat2d --bc periodic"; do
    t=$(echo $w | tr -d ' -')
    for f in 0 1; do
      NK_F0R=$f timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/ab_f0r2_${t}_$f.$r.log 2>&1
      echo "$w NK_F0R=$f round $r $(val gpurun_out/ab_f0r2_${t}_$f.$r.log)"
    done
  done
done
