# Whole-bench A/B of the streaming BLAS-1 grid cap (NK_RED_BLOCKS: 2048 blocks, the round-2 default,
# vs 16384 -- one or two 16-B elements per thread, the shape the stream probe streams fastest)
# plus the x-update kernel alone at both caps (GPU box)
set -e
mkdir -p gpurun_out
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels'];print(d['value'], {n: round(v['avg_us'],1) for n, v in k.items() if v['avg_us'] and n not in ('mgs_sweep','finalize')})" "$1"; }
for r in 1 2; do
  for w in "bratu2d" "heat2d"; do
    t=$(echo $w | tr -d ' -')
    for c in 2048 16384; do
      NK_RED_BLOCKS=$c timeout -k 10 250 python bench.py --workload $w --no-cpu-baseline > gpurun_out/ab_rb_${t}_$c.$r.log 2>&1
      echo "$w RED_BLOCKS=$c round $r $(val gpurun_out/ab_rb_${t}_$c.$r.log)"
    done
  done
done
for c in 2048 16384; do
  echo "kbench_upd NK_RED_BLOCKS=$c"
  NK_RED_BLOCKS=$c timeout -k 10 200 python tools/kbench_upd.py --rounds 3 --ks 1,3,11,30 --us 1,4
done
