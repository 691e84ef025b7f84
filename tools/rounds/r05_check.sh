#!/bin/bash
# Round-5 GPU check (run from the repo root): the -m gpu suite, then the PMC passes + bench lines of the
# workloads named in PROFILE_TAGS (tools/profile_round.sh).  A failing test (exit 1) does not stop the
# profiling; a crash, abort or time limit (any other non-zero status) ends the script there.
set -o pipefail
OUT=gpurun_out/r05_${1:-a}
mkdir -p "$OUT"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  echo "[r05] gpu suite"
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q ${PYTEST_ARGS:-} --timeout 300 --timeout-method thread > "$OUT/gputest.log" 2>&1
  rc=$?
  tail -n 3 "$OUT/gputest.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[r05] gpu suite ended with $rc: stopping"; exit $rc; fi
fi
if [ -n "${PROFILE_TAGS:-}" ]; then
  echo "[r05] profiles: $PROFILE_TAGS"
  PROFILE_PARTS="${PROFILE_PARTS:-pmc bench}" bash tools/profile_round.sh r05 quick || exit $?
fi
echo "[r05] done"
