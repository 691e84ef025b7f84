#!/bin/bash
# Whole-bench A/B of product-build variants (`make -C newtonkrylov.jl_amd variant TAG=... VDEFS=...`):
# LIBS="|w4|w5" ('' = lib/libnkhip.so, else lib/libnkhip_v_<tag>.so via NK_LIB_VARIANT), WL bench.py
# --workload arguments ('|'-separated), ROUNDS alternating rounds.  One line per run: matvecs/s and the
# kernels above 1 % of the time (average microseconds per launch).
set -e
cd "$(dirname "$0")/.."
B="timeout -k 10 240 python -u bench.py --no-cpu-baseline"
IFS='|' read -ra VS <<< "${LIBS:?}"
IFS='|' read -ra WLS <<< "${WL:-bratu2d}"
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for w in "${WLS[@]}"; do
    for v in "${VS[@]}"; do
      env NK_LIB_VARIANT=$v $B --workload $w > gpurun_out/ab_lib_run.log 2>&1
      r=$(tail -n 1 gpurun_out/ab_lib_run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k: round(v['avg_us'],1) for k, v in d['kernels'].items() if v.get('share',0) > 0.01})")
      echo "round $i [lib ${v:-product}] $w: $r"
    done
  done
done
