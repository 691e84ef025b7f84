#!/bin/bash
# same-box A/B of the product library at HEAD against an earlier build (_abold/, a git worktree of the
# commit the first round-3 bench lines came from): is a bench-line difference the code or the box?
set -e
cd "$(dirname "$0")/.."
for i in 1 2; do
  for t in _abold .; do
    for w in "--workload bratu2d" "--workload heat2d"; do
      (cd $t && timeout -k 10 300 python -u bench.py --no-cpu-baseline $w > /tmp/abh.log 2>&1)
      v=$(tail -n 1 /tmp/abh.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k: round(v['avg_us'],1) for k, v in list(d['kernels'].items())[:4]})")
      echo "round $i tree=$t $w: $v"
    done
  done
done
