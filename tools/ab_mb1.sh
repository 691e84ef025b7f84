# Cost of the cross-rank hand-off inside the resident sweep, measured on one GPU: a forced one-rank
# communicator whose every per-pass scalar goes through the peer mailbox (mb_send to itself + poll)
# against no communicator (GPU box): bash tools/ab_mb1.sh
set -e
mkdir -p gpurun_out
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels'];print(d['value'], d['config']['reductions'], round(k['mgs_sweep']['avg_us'],1), round(d['roofline']['avg_us'],1))" "$1"; }
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --prof-every 8 > gpurun_out/ab_mb1_local.$r.log 2>&1; echo "no communicator round $r $(val gpurun_out/ab_mb1_local.$r.log)"
  NK_DIST_FORCE=1 NK_DIST_MAILBOX=1 timeout -k 10 200 python bench.py --no-cpu-baseline --prof-every 8 > gpurun_out/ab_mb1_mb.$r.log 2>&1; echo "1-rank mailbox round $r $(val gpurun_out/ab_mb1_mb.$r.log)"
done
