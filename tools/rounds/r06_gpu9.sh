#!/bin/bash
# Round 6 (late): SURVEY §8e's strong scaling on 4096^2, rehearsed with 2 ranks on the box's GPU (each a
# 4096 x 2048 slab, resident sweeps on half the CUs each, ghost rows inside the Jv launch) -- the kernels of a
# 2-GPU strong-scaling run, time-sharing one GPU (not a scaling figure).
set -e -o pipefail
OUT=gpurun_out/r06_v
mkdir -p "$OUT"
if [[ " ${PARTS:-n2} " == *" n2 "* ]]; then
echo "[r06v] N=2 strong-scaling rehearsal (one 4096^2 problem)"
NK_RES_SHARED=1 NK_SHARED_FUSE_MAX=1073741824 timeout -k 10 400 python -u bench.py --gpus 2 --global-n 4096 \
    --transport mailbox --steps 3 --warmup 1 > "$OUT/rehearsal2_strong_bratu2d_4096.json" 2> "$OUT/rehearsal2_strong_bratu2d_4096.err"
fi
if [[ " ${PARTS:-} " == *" n48 "* ]]; then
  for n in 4 8; do
    echo "[r06v] N=$n strong-scaling rehearsal (one 4096^2 problem, ghost planes by the exchange kernel)"
    NK_RES_SHARED=1 GPU_MAX_HW_QUEUES=1 timeout -k 10 500 python -u bench.py --gpus $n --global-n 4096 \
        --transport mailbox --steps 3 --warmup 1 > "$OUT/rehearsal${n}_strong_bratu2d_4096.json" \
        2> "$OUT/rehearsal${n}_strong_bratu2d_4096.err"
  done
fi
echo "[r06v] done"
