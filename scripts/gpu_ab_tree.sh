#!/bin/bash
# same-box A/B of this tree against the baseline worktree ab_old/ (built in
# place): the bench line (no CPU legs) alternately, $1 rounds (default 2)
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
N=${1:-2}
for i in $(seq 1 $N); do
  for t in old new; do
    if [ $t = old ]; then B=ab_old/bench.py; else B=bench.py; fi
    timeout -k 10 300 python $B --no-cpu-baseline --steps 50 --warmup 10 ${BENCH_ARGS} > gpurun_out/ab_$t.json 2> gpurun_out/ab_$t.err || { tail -20 gpurun_out/ab_$t.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/ab_$t.json'));e=d.get('extras',{})
print('$t','C2',round(d['ms_per_step'],4),'C3',round(d.get('binary',{}).get('ms_per_step',0),4),'C4',round(e.get('lr_iteration',{}).get('ms_per_iteration',0),4),'C5',round(e.get('merge_sort',{}).get('ms_per_sort',0),2),'a2b',round(e.get('a2b',{}).get('ms_per_conversion',0),3))"
  done
done
