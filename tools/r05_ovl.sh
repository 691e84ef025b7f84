#!/bin/bash
# Overlapping wave tiles (k_st2d<..., OVL>, kbench NK_ST_OVL=1): the 2D parity tests on the variant, then
# whole-bench A/B against the per-row edge loads.  Stops at a crash / time limit.
set -o pipefail
OUT=gpurun_out/r05_ovl
mkdir -p "$OUT"
echo "[ovl] parity tests on the OVL variant"
NK_KBENCH_LIB=1 NK_ST_OVL=1 timeout -k 10 900 python -u -m pytest tests/test_hip.py tests/test_hip_schemes.py \
    tests/test_hip_f0r.py tests/test_hip_dist.py tests/test_hip_configs.py -m gpu -q --timeout 300 \
    --timeout-method thread > "$OUT/gputest_ovl.log" 2>&1
rc=$?
tail -n 3 "$OUT/gputest_ovl.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "[ovl] A/B"
VARIANTS="NK_ST_OVL=0|NK_ST_OVL=1" WL="${WL:-bratu2d|heat2d|heat2d --scheme trapezoid --bc periodic}" ROUNDS=2 \
    bash tools/ab_env.sh > "$OUT/ab_ovl.log" 2>&1 || exit $?
cat "$OUT/ab_ovl.log"
