# Resident-sweep arrival skew (tools/res_skew.py) at full / half / quarter residency, and at full
# residency with the slots interleaved across blocks (NK_RES_STRIDED=1): is the lateness of a block
# set by its XCD (blockIdx % 8) or by the addresses it streams?
set -e
cd $GRAFT_REPO_ROOT
run() {  # n rv [env...]
  n=$1; rv=$2; shift 2
  env "$@" NK_RES_TSTAMP=gpurun_out/ts_$n.bin timeout -k 10 120 python tools/kbench_res.py --n $n --ks 30 --rvs $rv --reps 2
  python tools/res_skew.py gpurun_out/ts_$n.bin 30
}
for n in ${SKEW_NS:-16777216 33554432 67108864}; do
  rv=1006; [ $n = 16777216 ] && rv=1000
  run $n $rv
done
if [ -n "$SKEW_STRIDED" ]; then echo "--- NK_RES_STRIDED=1"; run 16777216 1000 NK_RES_STRIDED=1; fi
