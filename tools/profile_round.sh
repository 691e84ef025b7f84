#!/bin/bash
# Regenerate one round's profiles on the GPU box (run from the repo root):
#     bash tools/profile_round.sh r01
# Results land in gpurun_out/prof_<round>/profiles/ (copy them to profiles/<round>/).
# Every GPU step has its own time limit; the script stops at the first failure.
#   1. rocprofv3 --kernel-trace --stats of the default bench         -> kernel_stats_bench.csv
#   2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) per workload  -> pmc_traffic_<workload>.json
#   3. the bench lines themselves (every workload tag, each with its CPU baseline)
#   4. in-process kernel-variant A/B (tools/kbench.py, tools/kbench_res.py)
set -e -o pipefail
R=${1:-r01}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$R
DST=$OUT/profiles  # only gpurun_out/ comes back from the box: copy to profiles/$R afterwards
mkdir -p "$OUT" "$DST"
export TMPDIR=/tmp

echo "[profile] kernel trace"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/bench_traced.log" 2>&1)
cp "$OUT/trace/run_kernel_stats.csv" "$DST/kernel_stats_bench.csv"
grep '^{"metric"' "$OUT/bench_traced.log" | tail -n 1 > "$DST/bench_under_rocprof.json"

echo "[profile] roctx ranges"
(cd /tmp && timeout -k 10 300 rocprofv3 --marker-trace --stats -d "$OUT/marker" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/bench_marker.log" 2>&1)
cp "$OUT/marker/run_marker_api_stats.csv" "$DST/marker_stats_bench.csv"

# workload tag -> bench.py arguments
declare -A WARGS=(
    [bratu2d]="--workload bratu2d"
    [heat2d]="--workload heat2d"
    [heat3d]="--workload heat3d"
    [heat2d_trapezoid_periodic]="--workload heat2d --scheme trapezoid --bc periodic"
    [heat3d_midpoint]="--workload heat3d --scheme midpoint"
)
TAGS="bratu2d heat2d heat3d heat2d_trapezoid_periodic heat3d_midpoint"

for w in $TAGS; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
        echo "[profile] $w $ctr"
        (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $ctr -d "$OUT/pmc_${w}_$ctr" -o run --output-format csv \
            -- python3 "$ROOT/bench.py" ${WARGS[$w]} --steps 1 --warmup 1 --itmax 60 --no-cpu-baseline --no-prof \
            > "$OUT/pmc_${w}_$ctr.log" 2>&1)
    done
    python3 tools/pmc_traffic.py "$OUT/pmc_${w}_FETCH_SIZE/run_counter_collection.csv" \
        "$OUT/pmc_${w}_WRITE_SIZE/run_counter_collection.csv" "$DST/pmc_traffic_$w.json"
done

echo "[profile] bench lines"
for w in $TAGS; do
    timeout -k 10 300 python3 bench.py ${WARGS[$w]} --traffic-json "$DST/pmc_traffic_$w.json" > "$OUT/bench_$w.log" 2>&1
    tail -n 1 "$OUT/bench_$w.log" > "$DST/bench_$w.json"
done
cp "$DST/bench_bratu2d.json" "$DST/bench.json"

echo "[profile] kernel variants"
timeout -k 10 300 python3 tools/kbench.py --rounds 3 --what mgs > "$DST/kbench_mgs.log" 2>&1
timeout -k 10 300 python3 tools/kbench.py --rounds 3 --what stencil > "$DST/kbench_stencil.log" 2>&1
timeout -k 10 300 python3 tools/kbench_res.py --ks 8,16,30 --rvs 0,32,48,64,89 > "$DST/kbench_res.log" 2>&1
echo "[profile] done"
