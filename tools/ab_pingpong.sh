#!/bin/bash
# the 2D stencil march as a ping-pong loop (no loaded register copied at the back edge) vs round 2's
# rotation (profiles/r02 numbers: heat2d euler residual 307.7 us, FD Jv+dot 626.4 us (F0R dotv 608.2),
# trapezoid periodic FD dotv 721.0 us, residual 317.1 us; Bratu FD Jv+dot 4096^2 129.0 us)
set -e
cd "$(dirname "$0")/.."
K="timeout -k 10 300 python -u tools/kbench_st.py --rounds 5 --reps 10 --rows 0"
$K --kinds 3 --side 8192 --modes 0:1,2:2 --fast 0,288
$K --kinds 7 --side 8192 --modes 2:2 --fast 416
$K --kinds 7 --side 8192 --modes 0:1 --fast 128
$K --kinds 5 --side 8192 --modes 0:1,2:2 --fast 0,288
$K --kinds 2 --side 4096 --modes 2:2,0:1 --fast 0,288
