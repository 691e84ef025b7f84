# Whole-bench A/B of resident-sweep defaults, alternating in one call (GPU box):  bash tools/ab_res.sh [what]
set -e
mkdir -p gpurun_out
B="timeout -k 10 200 python bench.py --no-cpu-baseline"
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d['value'])" "$1"; }
WHAT=${1:-all}
for r in 1 2; do
  if [ "$WHAT" = all ]; then
    for pre in 0 1; do NK_RES_PRE=$pre $B > gpurun_out/ab_b_pre$pre.$r.log 2>&1; echo "bratu2d 4096^2 NK_RES_PRE=$pre round $r $(val gpurun_out/ab_b_pre$pre.$r.log)"; done
    for nts in 0 1; do NK_RES_NTS=$nts $B --global-n 16384 --slab-of 8 > gpurun_out/ab_s_nts$nts.$r.log 2>&1; echo "config-4 slab NK_RES_NTS=$nts round $r $(val gpurun_out/ab_s_nts$nts.$r.log)"; done
    for nts in 0 1; do NK_RES_NTS=$nts $B --workload heat2d > gpurun_out/ab_h_nts$nts.$r.log 2>&1; echo "heat2d 8192^2 NK_RES_NTS=$nts round $r $(val gpurun_out/ab_h_nts$nts.$r.log)"; done
  fi
  for nts in 0 1; do NK_RES_NTS=$nts $B --workload heat3d > gpurun_out/ab_h3_nts$nts.$r.log 2>&1; echo "heat3d 512^3 NK_RES_NTS=$nts round $r $(val gpurun_out/ab_h3_nts$nts.$r.log)"; done
done
