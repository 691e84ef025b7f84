#!/bin/bash
# One GPU-box check of the current build (run from the repo root; results in gpurun_out/check_<tag>/):
# the -m gpu suite, smoke(), the bench as the driver runs it.  Each GPU step has its own time limit and
# the script stops at the first failure.
set -e -o pipefail
T=${1:-check}
OUT=gpurun_out/check_$T
mkdir -p "$OUT"
echo "[check] gpu suite"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gputest.log" 2>&1
tail -n 2 "$OUT/gputest.log"
echo "[check] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "[check] bench"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_driver_style.log" 2>&1
tail -n 1 "$OUT/bench_driver_style.log" > "$OUT/bench_driver_style.json"
python3 -c "import json; d=json.load(open('$OUT/bench_driver_style.json')); print(d['value'], d['roofline']['frac'])"
echo "[check] done"
