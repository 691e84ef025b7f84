#!/bin/bash
# Instruction counters per stencil kernel: rocprofv3 --pmc passes of SQ_INSTS_*
# (and the wave-state counters) over short bench runs of the workloads whose stencils sit below
# 0.70 of 8 TB/s, plus the Bratu FD Jv as the control.  Run from the repo root on the GPU box:
#     bash tools/pmc_insts.sh [tag ...]
# Results: gpurun_out/pmc_insts/<tag>_<pass>/run_counter_collection.csv; reduce them with
#     python tools/pmc_insts.py gpurun_out/pmc_insts > profiles/r04/pmc_insts.txt
# Only counters `rocprofv3 -L` lists are requested; each pass holds <= 8 SQ counters.
set -e -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_insts${PMC_SUFFIX:-}
mkdir -p "$OUT"
# PMC_EXPORT="NK_KBENCH_LIB=1 NK_ST_OVL=1": variables exported for the profiled runs (a kernel variant);
# exported before rocprofv3, never an `env` hop after its `--`
for kv in ${PMC_EXPORT:-}; do export "$kv"; done
export TMPDIR=/tmp
declare -A WARGS=(
    [bratu2d]="--workload bratu2d"
    [heat2d]="--workload heat2d"
    [heat2d_trapezoid_periodic]="--workload heat2d --scheme trapezoid --bc periodic"
    [heat3d_midpoint]="--workload heat3d --scheme midpoint"
    [heat3d_slab]="--workload heat3d --global-n 512 --slab-of 8"
    [heat3d_block]="--workload heat3d --global-n 512 --block-of 8"
)
TAGS=${*:-bratu2d heat2d_trapezoid_periodic heat2d heat3d_midpoint heat3d_slab}
(cd /tmp && timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1) || true
have() { grep -qw "$1" "$OUT/counters_list.txt"; }
pick() { local s=""; for c in "$@"; do if have "$c"; then s="$s $c"; fi; done; echo $s; }
PASS_A=$(pick SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES)
PASS_B=$(pick SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_BRANCH)
PASS_C=$(pick SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_FLAT)
echo "pass A: $PASS_A" | tee "$OUT/passes.txt"
echo "pass B: $PASS_B" | tee -a "$OUT/passes.txt"
echo "pass C: $PASS_C" | tee -a "$OUT/passes.txt"
for w in $TAGS; do
    for p in A B C; do
        eval "CTRS=\$PASS_$p"
        [ -n "$CTRS" ] || continue
        echo "[pmc_insts] $w pass $p"
        (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $CTRS -d "$OUT/${w}_$p" -o run --output-format csv \
            -- python3 "$ROOT/bench.py" ${WARGS[$w]} --steps 1 --warmup 1 --itmax 60 --no-cpu-baseline --no-prof \
            > "$OUT/${w}_$p.log" 2>&1)
    done
done
echo "[pmc_insts] done"
