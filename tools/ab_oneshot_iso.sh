set -e
K="timeout -k 10 300 python -u tools/kbench_st.py --rounds 7 --reps 10 --rows 0"
$K --kinds 2 --side 4096 --ny 4000 --modes 2:2,2:0 --fast 0,8192,262144
$K --kinds 2 --side 4096 --modes 2:2,2:0 --fast 0,8192,262144
$K --kinds 2 --side 4096 --ny 2000 --modes 2:2 --fast 0,8192,262144
