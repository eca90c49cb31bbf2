#!/bin/bash
# A/B of C3 / C4 / C5 under env variants given as "NAME=VALUE ..." arguments
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 ${ABC_ARGS} > gpurun_out/abc_$i.json 2> gpurun_out/abc_$i.err || exit $?
  python3 -c "
import json;d=json.load(open('gpurun_out/abc_$i.json'));e=d.get('extras',{})
print('$v','C2',round(d['ms_per_step'],4),'C3',round(d.get('binary',{}).get('ms_per_step',0),4),'C4',round(e.get('lr_iteration',{}).get('ms_per_iteration',0),4),'C5',round(e.get('merge_sort',{}).get('ms_per_sort',0),2))"
done
