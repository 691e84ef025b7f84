#!/bin/bash
# Round 6 (late): the in-launch exchanges with batched rounds (2D slab tiles: 2 elements per thread per round,
# 3D block tiles: 4) -- the distributed parity tests (both exchange forms bitwise), then the self-ring costs:
# 3D blocks in-launch (blocki) against the faces kernel (blocks), 2D Bratu slab fused against kernel.
set -e -o pipefail
OUT=gpurun_out/r06_g
mkdir -p "$OUT"
export TMPDIR=/tmp
P=" ${PARTS:-tests self} "
if [[ "$P" == *" tests "* ]]; then
  echo "[r06g] tests"
  timeout -k 10 900 python -u -m pytest tests/test_hip_dist.py -x -v --timeout 300 --timeout-method thread \
      > "$OUT/tests.log" 2>&1
fi
if [[ "$P" == *" self "* ]]; then
  echo "[r06g] 3D blocks: faces kernel vs in-launch"
  timeout -k 10 400 python -u tools/halo_self.py --nx 256 --ny 256 --nz 256 --modes mbox,blocks,blocki,mbox,blocks,blocki \
      > "$OUT/halo_self_blocks.log" 2>&1
  echo "[r06g] 2D Bratu 4096^2 slab: fused vs kernel"
  timeout -k 10 400 python -u tools/halo_self.py --nx 4096 --ny 4096 --nz 0 --modes mbox,fused,kernel,mbox,fused,kernel \
      > "$OUT/halo_self_2d.log" 2>&1
fi
echo "[r06g] done"
