#!/bin/bash
# Round 6: device-order GMRES parity, the in-launch 3D-block exchange (tests, then the config-5 block lines),
# the Infinity-Cache retention probe of the sweep, the block line's counters, the N=8 rehearsal.
# Every GPU step has its own limit; a failing step ends the call.
set -e -o pipefail
OUT=gpurun_out/r06_c
mkdir -p "$OUT"
export TMPDIR=/tmp
P=" ${PARTS:-tests lines nwc prof insts trace r8} "
if [[ "$P" == *" tests "* ]]; then
  echo "[r06] tests"
  timeout -k 10 900 python -u -m pytest tests/test_hip_devred.py tests/test_hip_dist.py -x -v --timeout 300 \
      --timeout-method thread -k "${TEST_K:-devred or self_block or blocks or form_is_rank_uniform}" > "$OUT/tests.log" 2>&1
fi
if [[ "$P" == *" lines "* ]]; then
  for pg in 2,2,2 1,2,4; do
    echo "[r06] block line $pg"
    timeout -k 10 300 python -u bench.py --workload heat3d --global-n 512 --block-of 8 --pgrid $pg --steps 3 --warmup 1 \
        > "$OUT/bench_block_$pg.json" 2> "$OUT/bench_block_$pg.err"
    NK_HALO_FUSE=0 timeout -k 10 300 python -u bench.py --workload heat3d --global-n 512 --block-of 8 --pgrid $pg --steps 3 \
        --warmup 1 > "$OUT/bench_block_${pg}_kernel.json" 2> "$OUT/bench_block_${pg}_kernel.err"
  done
fi
if [[ "$P" == *" nwc "* ]]; then
  echo "[r06] nwc"
  for r in 1 2; do
    for w in 128 96 64 32 0; do
      echo "round $r NK_RES_NWC=$w" >> "$OUT/nwc.log"
      NK_RES_NWC=$w timeout -k 10 120 python -u tools/kbench_res.py --n 16777216 --ks 30 --rvs 1000 --reps 5 >> "$OUT/nwc.log" 2>&1
    done
  done
fi
if [[ "$P" == *" prof "* ]]; then
  echo "[r06] pmc traffic of the block line"
  PROFILE_PARTS="pmc bench" PROFILE_TAGS="heat3d_block" bash tools/profile_round.sh r06 quick > "$OUT/prof.log" 2>&1
fi
if [[ "$P" == *" insts "* ]]; then
  echo "[r06] instruction counters"
  PMC_SUFFIX=_r06 bash tools/pmc_insts.sh heat3d_block heat3d_slab > "$OUT/insts.log" 2>&1
  python3 tools/pmc_insts.py gpurun_out/pmc_insts_r06 > "$OUT/pmc_insts_blocks.txt"
fi
if [[ "$P" == *" trace "* ]]; then
  echo "[r06] kernel trace of the block line"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/trace_block" -o run --output-format csv \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload heat3d --global-n 512 --block-of 8 --steps 3 \
      > "$GRAFT_REPO_ROOT/$OUT/bench_block_traced.log" 2>&1)
  cp "$OUT/trace_block/run_kernel_stats.csv" "$OUT/kernel_stats_heat3d_block.csv"
fi
if [[ "$P" == *" r8 "* ]]; then
  echo "[r06] 8-rank rehearsal of the N=8 SCALE command (4096^2 per rank)"
  GPU_MAX_HW_QUEUES=1 timeout -k 10 500 python -u bench.py --gpus 8 --transport mailbox --steps 2 --warmup 1 \
      > "$OUT/rehearsal8_bratu2d_4096.json" 2> "$OUT/rehearsal8_bratu2d_4096.err"
fi
echo "[r06] done"
