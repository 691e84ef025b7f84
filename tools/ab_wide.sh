# Whole-bench A/B of the wide streaming grid (NK_WIDE_BLOCKS=2048: the previous grid of the
# non-consumed streaming kernels, vs the default kRedCap - 2) on the three single-GPU workloads
set -e
mkdir -p gpurun_out
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels'];print(d['value'], d['calibration']['copy_gbs'], round(d['roofline']['frac_of_copy'],3), {n: round(v['avg_us'],1) for n, v in k.items() if v['avg_us'] and n in ('update_x','copy','fill','axpy')})" "$1"; }
for r in 1 2; do
  for w in "bratu2d" "heat2d" "heat3d"; do
    for c in 2048 d; do
      if [ $c = d ]; then timeout -k 10 250 python bench.py --workload $w --no-cpu-baseline > gpurun_out/ab_wide_${w}_$c.$r.log 2>&1
      else NK_WIDE_BLOCKS=$c timeout -k 10 250 python bench.py --workload $w --no-cpu-baseline > gpurun_out/ab_wide_${w}_$c.$r.log 2>&1; fi
      echo "$w WIDE=$c round $r $(val gpurun_out/ab_wide_${w}_$c.$r.log)"
    done
  done
done
