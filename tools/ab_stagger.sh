#!/bin/bash
# Vector start offsets (kbench NK_ALLOC_STAGGER=<bytes>: vector j's interior begins (j mod m) x that
# many bytes into its allocation, m = NK_ALLOC_STAGGER_MOD, 8; STAGGERS entries <bytes>[:m]) against the 2 MB-congruent default: the plain copy calibration and
# whole bench steps, rounds alternating (profiles/r03/ab_stagger.log)
set -e
cd "$(dirname "$0")/.."
B="timeout -k 10 240 python -u bench.py --no-cpu-baseline"
STAGGERS=${STAGGERS:-"0 256 4096 65536 0 1048576"}
WL=${WL:-"bratu2d|heat2d --scheme trapezoid --bc periodic|heat3d --scheme midpoint"}
IFS='|' read -ra WLS <<< "$WL"
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for w in "${WLS[@]}"; do
    for s in $STAGGERS; do
      m=8; [[ $s == *:* ]] && m=${s#*:}  # <bytes>[:<vectors per cycle>]
      NK_KBENCH_LIB=1 NK_ALLOC_STAGGER=${s%%:*} NK_ALLOC_STAGGER_MOD=$m $B --workload $w > gpurun_out/ab_stag.log 2>&1
      v=$(tail -n 1 gpurun_out/ab_stag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'copy', round(d.get('calibration',{}).get('copy_gbs',0)), {k: round(v['avg_us'],1) for k, v in d['kernels'].items() if v.get('share',0) > 0.01})")
      echo "round $i stagger=$s $w: $v"
    done
  done
done
