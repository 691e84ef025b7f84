#!/bin/bash
# Go/no-go bound for a run-ahead LDS ring in the resident sweep.  At full
# residency (4096^2: 128 slots per block = 89 register + 39 LDS) a ring must displace q slots from the
# LDS.  Cost side: the pass with the LDS holding 35 / 31 q slots (4 / 8 slots' room for a ring, the
# displaced slots streamed).  Benefit bound: the pass with NO hand-off at all (NK_RES_NOXCHG=1, wrong
# results, timing only) -- no run-ahead can save more than the whole wait.  (profiles/r03/ab_ring.log)
set -e
cd "$(dirname "$0")/.."
K="timeout -k 10 240 python -u tools/kbench_res.py --ks 16,30 --rvs 89 --reps 7"
echo "== default (rl = 39)"; $K
echo "== NK_RES_RL=35 (a 16 KB ring's room)"; NK_RES_RL=35 $K
echo "== NK_RES_RL=31 (a 32 KB ring's room)"; NK_RES_RL=31 $K
echo "== NK_RES_NOXCHG=1 (no hand-off: the bound of any run-ahead)"; NK_RES_NOXCHG=1 $K
