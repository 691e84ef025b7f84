#!/bin/bash
# Round 6, second GPU call: config 5's block line with its counters and the exact
# N=8 SCALE command rehearsed at its per-rank size with 8 ranks sharing the box's GPU (item 4).
set -e -o pipefail
OUT=gpurun_out/r06_b
mkdir -p "$OUT"
export TMPDIR=/tmp
if [[ " ${PARTS:-devred pg prof insts trace r8} " == *" devred "* ]]; then
  timeout -k 10 600 python -u -m pytest tests/test_hip_devred.py -x -v --timeout 300 --timeout-method thread \
      > "$OUT/devred.log" 2>&1
fi
if [[ " ${PARTS:-devred pg prof insts trace r8} " == *" pg "* ]]; then
  for pg in 2,2,2 1,2,4 1,1,8; do
    timeout -k 10 300 python -u bench.py --workload heat3d --global-n 512 --block-of 8 --pgrid $pg --steps 3 --warmup 1 \
        > "$OUT/bench_block_$pg.json" 2> "$OUT/bench_block_$pg.err"
  done
fi
if [[ " ${PARTS:-devred pg prof insts trace r8} " == *" prof "* ]]; then
  PROFILE_PARTS="pmc bench" PROFILE_TAGS="heat3d_block" bash tools/profile_round.sh r06 quick > "$OUT/prof.log" 2>&1
fi
if [[ " ${PARTS:-devred pg prof insts trace r8} " == *" insts "* ]]; then
  PMC_SUFFIX=_r06 bash tools/pmc_insts.sh heat3d_block heat3d_slab > "$OUT/insts.log" 2>&1
  python3 tools/pmc_insts.py gpurun_out/pmc_insts_r06 > "$OUT/pmc_insts_blocks.txt"
fi
if [[ " ${PARTS:-devred pg prof insts trace r8} " == *" trace "* ]]; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/trace_block" -o run --output-format csv \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload heat3d --global-n 512 --block-of 8 --steps 3 \
      > "$GRAFT_REPO_ROOT/$OUT/bench_block_traced.log" 2>&1)
  cp "$OUT/trace_block/run_kernel_stats.csv" "$OUT/kernel_stats_heat3d_block.csv"
fi
if [[ " ${PARTS:-devred pg prof insts trace r8} " == *" r8 "* ]]; then
  echo "[r06] 8-rank rehearsal of the N=8 SCALE command (4096^2 per rank)"
  GPU_MAX_HW_QUEUES=1 timeout -k 10 500 python -u bench.py --gpus 8 --transport mailbox --steps 2 --warmup 1 \
      > "$OUT/rehearsal8_bratu2d_4096.json" 2> "$OUT/rehearsal8_bratu2d_4096.err"
fi
echo "[r06] done"
