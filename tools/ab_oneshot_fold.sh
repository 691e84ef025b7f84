#!/bin/bash
# one-shot 8-row tiles with a dot epilogue: block partials handed on as they are (NK_TILE_PARTS=16382)
# vs folded in groups into about 1024 (the default) vs the row march (profiles/r03/ab_oneshot_fold.log)
set -e
cd "$(dirname "$0")/.."
for tp in 16382 1024; do
  echo "== NK_TILE_PARTS=$tp"
  NK_TILE_PARTS=$tp timeout -k 10 300 python -u tools/kbench_st.py --rounds 7 --reps 10 --rows 0 --kinds 2 --side 4096 --ny 4000 --modes 2:2 --fast 0,262144
  NK_TILE_PARTS=$tp timeout -k 10 300 python -u tools/kbench_st.py --rounds 7 --reps 10 --rows 0 --kinds 2 --side 4096 --ny 2000 --modes 2:2 --fast 0,262144
done
