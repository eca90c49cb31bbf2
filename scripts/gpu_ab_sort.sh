#!/bin/bash
# same-box A/B of the C5 sort (scripts/sort_timing.py) between the baseline
# tree ab_old/ and this tree, alternately: gpu_ab_sort.sh [rounds] [keys]
R=$GRAFT_REPO_ROOT
cd $R
N=${1:-2}
K=${2:-1048576}
for i in $(seq 1 $N); do
  for t in old new; do
    if [ $t = old ]; then D=ab_old; else D=.; fi
    r=$(timeout -k 10 200 python $D/scripts/sort_timing.py $K 3) || exit 1
    echo "$t $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["s_per_sort"]*1e3,2), "ms", d["ok"])')"
  done
done
