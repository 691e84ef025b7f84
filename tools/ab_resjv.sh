# Whole-bench A/B of the Jv fused into the resident sweep (NK_RES_JV=1) (GPU box): bash tools/ab_resjv.sh
set -e
mkdir -p gpurun_out
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels'];print(d['value'], {n:(v['launches'],round(v['avg_us'],1)) for n,v in list(k.items())[:4]})" "$1"; }
for r in 1 2; do
  for j in 0 1; do
    NK_RES_JV=$j timeout -k 10 200 python bench.py --no-cpu-baseline --prof-every 8 > gpurun_out/ab_resjv_$j.$r.log 2>&1; echo "NK_RES_JV=$j round $r $(val gpurun_out/ab_resjv_$j.$r.log)"
  done
done
