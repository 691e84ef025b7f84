#!/bin/bash
# Round-6 final measurement on one GPU box (run from the repo root), in parts that each fit one call:
#   PARTS="trace pmc bench" TAGS="..."  -> tools/profile_round.sh r06 (kernel stats of the default bench, PMC
#                                          FETCH / WRITE passes and the bench lines of the tags)
#   PARTS="r2"                         -> the N = 2 product path at full size on one GPU: two ranks of 4096^2
#                                          with resident sweeps on half the CUs each (NK_RES_SHARED=1) and the
#                                          ghost rows inside the Jv launch (NK_SHARED_FUSE_MAX) -- the kernels
#                                          of a 2-GPU run, time-sharing one GPU
# Results in gpurun_out/prof_r06/profiles/ and gpurun_out/r06_final/ (copied to profiles/r06/).
set -o pipefail
P=" ${PARTS:-trace pmc bench} "
if [[ "$P" == *" trace "* || "$P" == *" pmc "* || "$P" == *" bench "* ]]; then
  PROFILE_PARTS="$(echo $P | sed 's/r2//')" PROFILE_TAGS="${TAGS:-bratu2d}" bash tools/profile_round.sh r06 quick || exit $?
fi
if [[ "$P" == *" r2 "* ]]; then
  OUT=gpurun_out/r06_final
  mkdir -p "$OUT"
  echo "[r06] N=2 full-path rehearsal"
  NK_RES_SHARED=1 NK_SHARED_FUSE_MAX=1073741824 timeout -k 10 400 python -u bench.py --gpus 2 --transport mailbox \
      --steps 3 --warmup 1 > "$OUT/rehearsal2_fullpath_bratu2d_4096.json" 2> "$OUT/rehearsal2_fullpath_bratu2d_4096.err" || exit $?
fi
echo "[r06] final part done"
