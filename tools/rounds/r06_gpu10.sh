#!/bin/bash
# Round 6 (late): the packed-face exchange's grid size (kernel-variant build, NK_FACE_NB): 256 (the product's,
# one element per thread per face at 256^3) against 128 / 64 / 32 blocks, self ring, 256^3 block.
set -e -o pipefail
OUT=gpurun_out/r06_w
mkdir -p "$OUT"
for nb in 256 64 128 32 256; do
  echo "[r06w] NK_FACE_NB=$nb"
  echo "== NK_FACE_NB=$nb" >> "$OUT/face_nb.log"
  NK_KBENCH_LIB=1 NK_FACE_NB=$nb timeout -k 10 300 python -u tools/halo_self.py --nx 256 --ny 256 --nz 256 \
      --modes blocks >> "$OUT/face_nb.log" 2>&1
done
echo "[r06w] done"
