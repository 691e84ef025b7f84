# The 2D stencil with raw rows three ahead (NK_ST_D3 / fast bit 64) against two ahead: kernel bench,
# whole-bench A/B, and the 2D stencil parity tests forced onto the D3 kernels (GPU box)
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/kbench_st.py --kinds 2,3 --side 4096 --fast 0,64 --rows 0 --modes 2:2,0:1,2:1 > gpurun_out/d3_kbench_4096.log 2>&1
timeout -k 10 200 python -u tools/kbench_st.py --kinds 3,5 --side 8192 --fast 0,64,32,96 --rows 0 --modes 2:2,0:1 > gpurun_out/d3_kbench_8192.log 2>&1
NK_ST_D3=1 timeout -k 10 400 python -u -m pytest tests/test_hip.py tests/test_hip_schemes.py tests/test_hip_f0r.py tests/test_hip_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/d3_tests.log 2>&1
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels'];print(d['value'], {n: round(v['avg_us'],1) for n, v in k.items() if v['avg_us'] and n.startswith(('jv','resid'))})" "$1"; }
for r in 1 2; do
  for w in bratu2d heat2d; do
    for c in 0 1; do
      NK_ST_D3=$c timeout -k 10 250 python bench.py --workload $w --no-cpu-baseline > gpurun_out/ab_d3_${w}_$c.$r.log 2>&1
      echo "$w D3=$c round $r $(val gpurun_out/ab_d3_${w}_$c.$r.log)"
    done
  done
done
