#!/bin/bash
# Round 6: block parity / form tests and the multi-rank device-order GMRES tests, then the config-5 block
# line with the one-slot x edges, against the 4-wave-cap variant build (NK_LIB_VARIANT=blkcap), interleaved.
set -e -o pipefail
OUT=gpurun_out/r06_e
mkdir -p "$OUT"
export TMPDIR=/tmp
P=" ${PARTS:-tests lines} "
if [[ "$P" == *" tests "* ]]; then
  echo "[r06] tests"
  timeout -k 10 1200 python -u -m pytest tests/test_hip_dist.py -x -v --timeout 300 --timeout-method thread \
      -k "${TEST_K:-self_block or blocks_match or budget or eight_ranks_256}" > "$OUT/tests.log" 2>&1
fi
if [[ "$P" == *" lines "* ]]; then
  for r in 1 2; do
    for v in "" blkcap; do
      echo "[r06] block line ${v:-product} round $r"
      NK_LIB_VARIANT=$v timeout -k 10 300 python -u bench.py --workload heat3d --global-n 512 --block-of 8 --steps 3 \
          --warmup 1 --no-cpu-baseline > "$OUT/bench_block_${v:-product}_$r.json" 2> "$OUT/bench_block_${v:-product}_$r.err"
    done
  done
fi
echo "[r06] done"
