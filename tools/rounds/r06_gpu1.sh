#!/bin/bash
# Round 6, first GPU call: the refactored build's GPU suite subset (dist + new form test), the config-5
# block line (bench.py --block-of 8), and the 8-rank 256^3 z-slab rehearsal that stalled in r05 -- at
# the DEFAULT mailbox spin limit, so a stall errors instead of running 30 s per step.
set -e -o pipefail
OUT=gpurun_out/r06_a
mkdir -p "$OUT"
echo "[r06] tests"
timeout -k 10 900 python -u -m pytest tests/test_hip_dist.py -x -v --timeout 300 --timeout-method thread \
    -k "${TEST_K:-form_is_rank_uniform or zslabs or blocks_match}" > "$OUT/tests.log" 2>&1
echo "[r06] block line"
timeout -k 10 300 python -u bench.py --workload heat3d --global-n 512 --block-of 8 --steps 3 --warmup 1 \
    > "$OUT/bench_block.json" 2> "$OUT/bench_block.err"
echo "[r06] 8-rank 256^3 z-slab rehearsal (default spin limit)"
export GPU_MAX_HW_QUEUES=1
timeout -k 10 400 python -u bench.py --gpus 8 --transport mailbox --workload heat3d --global-n 256 \
    --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/rehearsal8_heat3d_256_slabs.json" 2> "$OUT/rehearsal8_heat3d_256_slabs.err"
echo "[r06] done"
