set -e
mkdir -p gpurun_out
B="timeout -k 10 200 python bench.py --no-cpu-baseline"
for r in 1 2; do
  for pre in 0 1; do NK_RES_PRE=$pre $B > gpurun_out/ab_b_pre$pre.$r.log 2>&1; echo "bratu pre=$pre $(python -c "import json;d=json.loads(open('gpurun_out/ab_b_pre$pre.$r.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['avg_us'])")"; done
  for nts in 0 1; do NK_RES_NTS=$nts $B --global-n 16384 --slab-of 8 > gpurun_out/ab_s_nts$nts.$r.log 2>&1; echo "slab nts=$nts $(python -c "import json;d=json.loads(open('gpurun_out/ab_s_nts$nts.$r.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['avg_us'])")"; done
  for nts in 0 1; do NK_RES_NTS=$nts $B --workload heat2d > gpurun_out/ab_h_nts$nts.$r.log 2>&1; echo "heat2d nts=$nts $(python -c "import json;d=json.loads(open('gpurun_out/ab_h_nts$nts.$r.log').read().strip().splitlines()[-1]);print(d['value'], d['kernels']['mgs_sweep']['avg_us'])")"; done
done
timeout -k 10 400 python -u -m pytest tests/test_hip_resident.py tests/test_hip_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/restests.log 2>&1
tail -2 gpurun_out/restests.log
