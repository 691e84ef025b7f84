#!/bin/bash
# Regenerate one round's profiles on the GPU box (run from the repo root):
#     bash tools/profile_round.sh r03 [quick]
# Results land in gpurun_out/prof_<round>/profiles/ (copy them to profiles/<round>/).
# Every GPU step has its own time limit; the script stops at the first failure.
#   1. rocprofv3 --kernel-trace --stats of the default bench         -> kernel_stats_bench.csv
#   2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) per workload  -> pmc_traffic_<tag>_<side>.json
#      (bench.py applies a PMC file only to the workload AND size it was measured on)
#   3. the bench lines themselves (every workload tag; CPU baseline on the default sizes)
#   4. (not with "quick") in-process kernel-variant A/B (tools/kbench.py, tools/kbench_res.py)
# PROFILE_PARTS="trace pmc bench" and PROFILE_TAGS="bratu2d heat2d ..." select a subset (one gpurun
# call stays well inside its time limit).
set -e -o pipefail
R=${1:-r03}
MODE=${2:-full}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$R
DST=$OUT/profiles  # only gpurun_out/ comes back from the box: copy to profiles/$R afterwards
mkdir -p "$OUT" "$DST"
export TMPDIR=/tmp

PARTS=${PROFILE_PARTS:-trace pmc bench}
if [[ " $PARTS " == *" trace "* ]]; then
echo "[profile] kernel trace"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/bench_traced.log" 2>&1)
cp "$OUT/trace/run_kernel_stats.csv" "$DST/kernel_stats_bench.csv"
grep '^{"metric"' "$OUT/bench_traced.log" | tail -n 1 > "$DST/bench_under_rocprof.json"
fi

# workload tag -> bench.py arguments, and the size part of its PMC file name (W.side in bench.py)
declare -A WARGS=(
    [bratu2d]="--workload bratu2d"
    [heat2d]="--workload heat2d"
    [heat3d]="--workload heat3d"
    [heat2d_trapezoid_periodic]="--workload heat2d --scheme trapezoid --bc periodic"
    [heat3d_midpoint]="--workload heat3d --scheme midpoint"
    [bratu2d_slab]="--workload bratu2d --global-n 16384 --slab-of 8"
    [heat3d_slab]="--workload heat3d --global-n 512 --slab-of 8"
    [heat3d_block]="--workload heat3d --global-n 512 --block-of 8"
)
declare -A WFILE=(
    [bratu2d]="bratu2d_4096" [heat2d]="heat2d_8192" [heat3d]="heat3d_512"
    [heat2d_trapezoid_periodic]="heat2d_trapezoid_periodic_8192" [heat3d_midpoint]="heat3d_midpoint_512"
    [bratu2d_slab]="bratu2d_16384x2048" [heat3d_slab]="heat3d_512x64" [heat3d_block]="heat3d_block256x256x256"
)
TAGS=${PROFILE_TAGS:-bratu2d heat2d heat3d heat2d_trapezoid_periodic heat3d_midpoint bratu2d_slab heat3d_slab}

if [[ " $PARTS " == *" pmc "* ]]; then
for w in $TAGS; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
        echo "[profile] $w $ctr"
        (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $ctr -d "$OUT/pmc_${w}_$ctr" -o run --output-format csv \
            -- python3 "$ROOT/bench.py" ${WARGS[$w]} --steps 1 --warmup 1 --itmax 60 --no-cpu-baseline --no-prof \
            > "$OUT/pmc_${w}_$ctr.log" 2>&1)
    done
    python3 tools/pmc_traffic.py "$OUT/pmc_${w}_FETCH_SIZE/run_counter_collection.csv" \
        "$OUT/pmc_${w}_WRITE_SIZE/run_counter_collection.csv" "$DST/pmc_traffic_${WFILE[$w]}.json"
done
fi

if [[ " $PARTS " == *" bench "* ]]; then
echo "[profile] bench lines"
for w in $TAGS; do
    TJ="$DST/pmc_traffic_${WFILE[$w]}.json"
    [ -f "$TJ" ] || TJ="profiles/$R/pmc_traffic_${WFILE[$w]}.json"  # PMC passes of an earlier call
    timeout -k 10 300 python3 bench.py ${WARGS[$w]} --traffic-json "$TJ" \
        > "$OUT/bench_$w.log" 2>&1
    tail -n 1 "$OUT/bench_$w.log" > "$DST/bench_$w.json"
done
[ -f "$DST/bench_bratu2d.json" ] && cp "$DST/bench_bratu2d.json" "$DST/bench.json"
fi

if [ "$MODE" = full ]; then
    echo "[profile] kernel variants"
    timeout -k 10 300 python3 tools/kbench.py --rounds 3 --what mgs > "$DST/kbench_mgs.log" 2>&1
    timeout -k 10 300 python3 tools/kbench.py --rounds 3 --what stencil > "$DST/kbench_stencil.log" 2>&1
    timeout -k 10 300 python3 tools/kbench_res.py --ks 8,16,30 --rvs 0,32,48,64,89 > "$DST/kbench_res.log" 2>&1
fi
echo "[profile] done"
