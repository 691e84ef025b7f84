# Partial residency: the first NK_RES_NTC streamed slots of each block load V_{i+1} cached (so the next
# pass re-reads them from the Infinity Cache), the rest non-temporal; per pass (tools/kbench_res.py,
# default variant) at half / a quarter / an eighth resident (GPU box): bash tools/ab_ntc.sh [values]
set -e
for n in ${NTC_NS:-33554432 67108864 134217728}; do
  for c in ${1:-0 80 96 112 128}; do
    echo "NK_RES_NTC=$c n=$n"
    NK_RES_NTC=$c timeout -k 10 150 python tools/kbench_res.py --n $n --ks 30 --rvs 1006 --reps 3
  done
done
