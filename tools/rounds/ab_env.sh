#!/bin/bash
# Whole-bench A/B of kernel-variant knobs (kbench build): VARIANTS="A=1 B=2|A=0" (one environment per
# '|'-separated entry), WL="bratu2d|heat2d --scheme trapezoid" (bench.py --workload arguments), ROUNDS
# alternating rounds.  One line per run: matvecs/s, copy calibration, the kernels above 1 % of the time.
set -e
cd "$(dirname "$0")/.."
B="timeout -k 10 240 python -u bench.py --no-cpu-baseline"
IFS='|' read -ra VS <<< "${VARIANTS:?}"
IFS='|' read -ra WLS <<< "${WL:-bratu2d}"
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for w in "${WLS[@]}"; do
    for v in "${VS[@]}"; do
      env NK_KBENCH_LIB=1 $v $B --workload $w > gpurun_out/ab_env_run.log 2>&1
      r=$(tail -n 1 gpurun_out/ab_env_run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'copy', round(d.get('calibration',{}).get('copy_gbs',0)), {k: round(v['avg_us'],1) for k, v in d['kernels'].items() if v.get('share',0) > 0.01})")
      echo "round $i [$v] $w: $r"
    done
  done
done
