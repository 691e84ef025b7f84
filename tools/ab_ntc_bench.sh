# Whole-bench A/B of the cached streamed slots (NK_RES_NTC=0: every streamed V_{i+1} non-temporal, vs
# the default room-filling count) on the partly resident workloads (GPU box)
set -e
mkdir -p gpurun_out
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels'];print(d['value'], round(k['mgs_sweep']['avg_us'],1))" "$1"; }
for r in 1 2; do
  for w in "bratu2d --global-n 16384 --slab-of 8" "heat2d" "heat3d"; do
    t=$(echo $w | tr -d ' -')
    for c in 0 d; do
      if [ $c = 0 ]; then NK_RES_NTC=0 timeout -k 10 250 python bench.py --workload $w --no-cpu-baseline > gpurun_out/ab_ntcb_${t}_$c.$r.log 2>&1
      else timeout -k 10 250 python bench.py --workload $w --no-cpu-baseline > gpurun_out/ab_ntcb_${t}_$c.$r.log 2>&1; fi
      echo "$w NTC=$c round $r $(val gpurun_out/ab_ntcb_${t}_$c.$r.log)"
    done
  done
done
