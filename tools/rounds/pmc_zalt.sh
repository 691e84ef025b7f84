#!/bin/bash
# FETCH_SIZE of the 3D FD Jv under each tile order (kbench NK_ST3_ZALT 0 / 1 / 3): did the z-halo
# sharing cut the traffic, and did that buy time?  (profiles/r03/pmc_zalt.log; timing in ab_zalt2.log)
set -e -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_zalt
mkdir -p "$OUT"
export TMPDIR=/tmp
for z in 0 1 3; do
  for k in "6 256" "4 288"; do
    set -- $k
    echo "[pmc_zalt] kind $1 fast $2 zalt $z"
    (cd /tmp && NK_ST3_ZALT=$z timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/z${z}_k$1" -o run --output-format csv \
        -- python3 "$ROOT/tools/kbench_st.py" --rounds 1 --reps 5 --rows 0 --kinds $1 --side 512 --modes 2:2 --fast $2 \
        > "$OUT/z${z}_k$1.log" 2>&1)
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/z*_k*/run_counter_collection.csv")):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE" and "k_st3l" in r["Kernel_Name"]:
            acc[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(2.0 * 1024.0 * float(r["Counter_Value"]))
    for k, v in acc.items():
        print(f"{os.path.basename(os.path.dirname(f)):8s} {k:60s} n={len(v):3d} fetch/launch {sum(v) / len(v) / 1e6:9.1f} MB")
PY
