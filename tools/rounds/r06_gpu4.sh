#!/bin/bash
# Round 6: the block parity tests in both exchange forms, then config 5's block line (default form) with its
# PMC traffic, instruction counters and kernel trace, and the headline bench (CPU baseline in device order:
# the agreement's x bit for bit).
set -e -o pipefail
OUT=gpurun_out/r06_d
mkdir -p "$OUT"
export TMPDIR=/tmp
P=" ${PARTS:-tests prof insts trace bench} "
if [[ "$P" == *" tests "* ]]; then
  echo "[r06] tests"
  timeout -k 10 900 python -u -m pytest tests/test_hip_dist.py -x -v --timeout 300 --timeout-method thread \
      -k "${TEST_K:-self_block or blocks_match}" > "$OUT/tests.log" 2>&1
fi
if [[ "$P" == *" prof "* ]]; then
  echo "[r06] pmc traffic of the block line"
  PROFILE_PARTS="pmc bench" PROFILE_TAGS="heat3d_block" bash tools/profile_round.sh r06 quick > "$OUT/prof.log" 2>&1
fi
if [[ "$P" == *" insts "* ]]; then
  echo "[r06] instruction counters"
  PMC_SUFFIX=_r06d bash tools/pmc_insts.sh heat3d_block heat3d_slab > "$OUT/insts.log" 2>&1
  python3 tools/pmc_insts.py gpurun_out/pmc_insts_r06d > "$OUT/pmc_insts_blocks.txt"
fi
if [[ "$P" == *" trace "* ]]; then
  echo "[r06] kernel trace of the block line"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/trace_block" -o run --output-format csv \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload heat3d --global-n 512 --block-of 8 --steps 3 \
      > "$GRAFT_REPO_ROOT/$OUT/bench_block_traced.log" 2>&1)
  cp "$OUT/trace_block/run_kernel_stats.csv" "$OUT/kernel_stats_heat3d_block.csv"
fi
if [[ "$P" == *" bench "* ]]; then
  echo "[r06] headline bench"
  timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
fi
echo "[r06] done"
