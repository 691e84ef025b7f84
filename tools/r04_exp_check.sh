#!/bin/bash
# Round-4 GPU check of the shared correctly rounded exp (run from the repo root on the GPU box):
# the exp / core parity tests, tools/bratu_parity_probe.py, the default bench, and a whole-bench A/B of
# nk_exp against the platform exp (kbench NK_EXP_OCML).  Results in gpurun_out/r04_exp/.
# Test failures (pytest rc 1) do not stop the script; a timeout, abort or fault does.
set -o pipefail
OUT=gpurun_out/r04_exp
mkdir -p $OUT
step() {  # step NAME SECONDS CMD...: run with a time limit; stop on anything but success / test failures
    local name=$1 secs=$2
    shift 2
    echo "[r04] $name"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[r04] $name rc=$rc"
    tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step gputest 900 python -u -m pytest ${TESTS:-tests/test_hip_exp.py tests/test_hip.py} -v --timeout 300 --timeout-method thread
step probe 300 python -u tools/bratu_parity_probe.py
step bench 300 python -u bench.py --steps 20 --warmup 5
tail -n 1 $OUT/bench.log > $OUT/bench.json
if [ "${AB:-1}" = 1 ]; then
    VARIANTS="${AB_VARIANTS:-NK_EXP_OCML=0|NK_EXP_OCML=1}" WL="${AB_WL:-bratu2d}" ROUNDS=${AB_ROUNDS:-2} step ab_exp 900 bash tools/ab_env.sh
fi
echo "[r04] done"
