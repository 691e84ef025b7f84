#!/bin/bash
# Counter passes over tools/probe.py (one kernel configuration, several launches): occupancy,
# wait/issue split and L2 hit rate of the FD Jv and MGS kernels.  Run from the repo root on the box.
set -e -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_probe
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr TA_BUSY_max" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
    i=$((i + 1))
    (cd /tmp && timeout -k 10 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv \
        -- python3 "$ROOT/tools/probe.py" ${1:-both} > "$OUT/p$i.log" 2>&1) || echo "pass $i ($set) failed"
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("nk::(anonymous namespace)::", "").split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}")
PY
