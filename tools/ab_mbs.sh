# Cross-rank hand-off of the resident sweep with 1 vs 8 sending blocks (NK_MB_SENDERS), on one GPU
# through a forced one-rank communicator (every per-pass scalar goes through the peer mailbox)
# (GPU box): bash tools/ab_mbs.sh
set -e
mkdir -p gpurun_out
val() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels'];print(d['value'], d['config']['reductions'], round(k['mgs_sweep']['avg_us'],1))" "$1"; }
for r in 1 2 3; do
  for s in 1 8; do
    NK_MB_SENDERS=$s NK_DIST_FORCE=1 NK_DIST_MAILBOX=1 timeout -k 10 200 python bench.py --no-cpu-baseline --prof-every 8 > gpurun_out/ab_mbs.$s.$r.log 2>&1
    echo "senders $s round $r $(val gpurun_out/ab_mbs.$s.$r.log)"
  done
done
