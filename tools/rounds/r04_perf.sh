#!/bin/bash
# Round-4 performance evidence (run from the repo root on the GPU box; results in gpurun_out/r04_perf/):
#   halo    tools/halo_cost.py's 2-rank 512x128x64 GMRES on one shared GPU
#   ym      tools/kbench_cmp.py (y-march outputs vs the z-march's; the reductions differ in order) and
#           tools/kbench_ym.py: 3D y-march vs z-march per rows-per-chunk
#   pmc     tools/pmc_insts.sh instruction counters per stencil
# STEPS selects ("halo ym pmc" by default).  A timeout, abort or fault ends the script.
set -o pipefail
OUT=gpurun_out/r04_perf
mkdir -p $OUT
step() {
    local name=$1 secs=$2
    shift 2
    echo "[r04p] $name"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[r04p] $name rc=$rc"
    tail -n 4 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
for s in ${STEPS:-halo ym pmc}; do
    case $s in
    halo) step halo 300 python -u tools/halo_cost.py --nx 512 --ny 128 --nzl 64 --itmax 40 --reps 20 --modes alone,fused ;;
    ym)
        step ym_cmp 240 python -u tools/kbench_cmp.py --cases ${YM_CASES:-4:512:64:2:2:0:524288,4:512:64:0:1:0:524288,6:512:64:2:2:0:524288,8:512:64:2:2:0:524288,4:200:9:1:2:0:524288,8:128:16:2:2:128:524416,6:512:64:2:2:256:524544,4:512:64:2:2:32:524320}
        for r in ${YM_ROWS:-32 64 128}; do
            NK_ST3Y_ROWS=$r step ym_$r 240 python -u tools/kbench_ym.py --rounds 3
        done ;;
    pmc) step pmc 900 bash tools/pmc_insts.sh ${PMC_TAGS:-} && python tools/pmc_insts.py gpurun_out/pmc_insts > $OUT/pmc_insts.txt ;;
    esac
done
echo "[r04p] done"
