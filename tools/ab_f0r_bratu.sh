# Whole-bench A/B: the 2D Bratu FD operator reading F0 (NK_F0R=1, default: heat kinds only recompute)
# vs recomputing F(u) with its second exp (NK_F0R=2), with the current 2D tile rule (GPU box)
set -e
mkdir -p gpurun_out
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels'];j={n:round(v['avg_us'],1) for n,v in k.items() if n.startswith('jv_fd')};print(d['value'], j)" "$1"; }
for r in 1 2 3; do
  for w in "bratu2d" "bratu2d --global-n 16384 --slab-of 8"; do
    t=$(echo $w | tr -d ' -')
    for f in 1 2; do
      NK_F0R=$f timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --prof-every 8 > gpurun_out/ab_f0rb_${t}_$f.$r.log 2>&1
      echo "$w NK_F0R=$f round $r $(val gpurun_out/ab_f0rb_${t}_$f.$r.log)"
    done
  done
done
