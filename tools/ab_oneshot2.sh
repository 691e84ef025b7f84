#!/bin/bash
# The product's one-shot LDS tiles for the FD operator (k_st2t, 8 rows, group-folded partials) vs the
# row march it replaced (kbench fast bit 262144 / NK_ST_ONESHOT=0): per kernel class at the bench sizes,
# then whole bench steps alternating (profiles/r03/ab_oneshot2.log)
set -e
cd "$(dirname "$0")/.."
K="timeout -k 10 300 python -u tools/kbench_st.py --rounds 7 --reps 10 --rows 0"
$K --kinds 2 --side 4096 --modes 2:2,2:3 --fast 0,262144
$K --kinds 2 --side 4096 --modes 2:2 --fast 288,262432
$K --kinds 3 --side 8192 --modes 2:2 --fast 288,262432,256,262400
$K --kinds 7 --side 8192 --modes 2:2 --fast 256,262400
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
for i in 1 2; do
  for o in 0 1; do
    for w in "--workload bratu2d" "--workload heat2d" "--workload heat2d --scheme trapezoid --bc periodic"; do
      NK_KBENCH_LIB=1 NK_ST_ONESHOT=$o $B $w > /tmp/ab_os.log 2>&1
      v=$(tail -n 1 /tmp/ab_os.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k: round(v['avg_us'],1) for k, v in d['kernels'].items() if k.startswith('jv')})")
      echo "round $i oneshot=$o $w: $v"
    done
  done
done
