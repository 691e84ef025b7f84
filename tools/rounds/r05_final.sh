#!/bin/bash
# Round-5 final measurement on one GPU box (run from the repo root), every GPU step under its own limit:
#   1. rocprofv3 --kernel-trace --stats of the default bench (-> kernel_stats_bench.csv)
#   2. PMC FETCH/WRITE passes + bench lines of every workload (tools/profile_round.sh)
# Results in gpurun_out/prof_r05/profiles/ (copy to profiles/r05/).
set -o pipefail
PARTS=${PARTS:-trace pmc bench}
TAGS=${TAGS:-bratu2d heat2d heat3d heat2d_trapezoid_periodic heat3d_midpoint bratu2d_slab heat3d_slab}
PROFILE_PARTS="$PARTS" PROFILE_TAGS="$TAGS" bash tools/profile_round.sh r05 quick
