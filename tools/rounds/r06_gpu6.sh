#!/bin/bash
# Round 6 (late): the exchange kernels with their load batches ahead of the stores (k_faces_ipc, k_halo_ipc):
# the distributed parity tests, the config-5 block lines (faces launch time), a slab line on the exchange
# kernel, the block line's kernel trace.  Every GPU step has its own limit; a failing step ends the call.
set -e -o pipefail
OUT=gpurun_out/r06_f
mkdir -p "$OUT"
export TMPDIR=/tmp
P=" ${PARTS:-tests lines trace} "
if [[ "$P" == *" tests "* ]]; then
  echo "[r06f] tests"
  timeout -k 10 900 python -u -m pytest tests/test_hip_dist.py -x -v --timeout 300 --timeout-method thread \
      > "$OUT/tests.log" 2>&1
fi
if [[ "$P" == *" lines "* ]]; then
  for pg in 2,2,2 1,2,4; do
    echo "[r06f] block line $pg"
    timeout -k 10 300 python -u bench.py --workload heat3d --global-n 512 --block-of 8 --pgrid $pg --steps 3 --warmup 1 \
        > "$OUT/bench_block_$pg.json" 2> "$OUT/bench_block_$pg.err"
  done
  echo "[r06f] self-ring exchange costs (slab: fused / kernel; 256^3 block: faces kernel)"
  timeout -k 10 400 python -u tools/halo_self.py --nx 512 --ny 512 --nz 64 --modes plain,mbox,fused,kernel,plain,mbox,fused,kernel \
      > "$OUT/halo_self_slab.log" 2>&1
  timeout -k 10 400 python -u tools/halo_self.py --nx 256 --ny 256 --nz 256 --modes plain,mbox,blocks,plain,mbox,blocks \
      > "$OUT/halo_self_blocks.log" 2>&1
fi
if [[ "$P" == *" trace "* ]]; then
  echo "[r06f] kernel trace of the block line"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/trace_block" -o run --output-format csv \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload heat3d --global-n 512 --block-of 8 --steps 3 \
      > "$GRAFT_REPO_ROOT/$OUT/bench_block_traced.log" 2>&1)
  cp "$OUT/trace_block/run_kernel_stats.csv" "$OUT/kernel_stats_heat3d_block.csv"
fi
echo "[r06f] done"
