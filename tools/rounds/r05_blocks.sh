#!/bin/bash
# Round 5: 3D blocks on the GPU box -- the block parity / bench tests, then config 5 (512^3 heat3d) on
# 8 ranks sharing the box's one GPU over the mailbox: z-slabs against 2x2x2 blocks (a rehearsal: the
# ranks time-share one GPU, so the aggregate rate compares the decompositions, not 8 GPUs).
set -e -o pipefail
OUT=gpurun_out/r05_blocks${1:+_$1}
mkdir -p "$OUT"
[ -n "$NO_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_hip_dist.py tests/test_bench_launcher.py -x -v --timeout 300 \
    --timeout-method thread -k "${TEST_K:-blocks or block_bench or two_rank_bench}" > "$OUT/tests.log" 2>&1
export GPU_MAX_HW_QUEUES=1
# time-shared ranks: a rank's reduction partner may be descheduled for seconds -- a long poll limit
export NK_MB_SPIN_LIMIT=${NK_MB_SPIN_LIMIT:-1073741824}
for pg in "" auto; do
    tag=${pg:-slabs}
    echo "[r05_blocks] config 5 rehearsal $tag"
    timeout -k 10 400 python -u bench.py --gpus 8 --transport mailbox --workload heat3d --global-n ${GN:-512} \
        ${pg:+--pgrid $pg} --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_c5_$tag.json" 2> "$OUT/bench_c5_$tag.err"
done
echo "[r05_blocks] done"
