#!/bin/bash
# Round 6 (late): the N > 1 product paths after the exchange changes -- the N = 2 full path on one GPU (resident
# sweeps on half the CUs each, ghost rows inside the Jv launch through halo_tile_exchange's batched rounds) and
# the N = 8 SCALE command with 8 ranks on the box's GPU (ghost planes through k_halo_ipc).
set -e -o pipefail
OUT=gpurun_out/r06_s
mkdir -p "$OUT"
echo "[r06s] N=2 full-path rehearsal"
NK_RES_SHARED=1 NK_SHARED_FUSE_MAX=1073741824 timeout -k 10 400 python -u bench.py --gpus 2 --transport mailbox \
    --steps 3 --warmup 1 > "$OUT/rehearsal2_fullpath_bratu2d_4096.json" 2> "$OUT/rehearsal2_fullpath_bratu2d_4096.err"
echo "[r06s] N=8 rehearsal (4096^2 per rank, 8 ranks on one GPU)"
GPU_MAX_HW_QUEUES=1 timeout -k 10 500 python -u bench.py --gpus 8 --transport mailbox --steps 2 --warmup 1 \
    > "$OUT/rehearsal8_bratu2d_4096.json" 2> "$OUT/rehearsal8_bratu2d_4096.err"
echo "[r06s] done"
