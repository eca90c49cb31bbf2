#!/bin/bash
# k_digits kernel stats of the C2 job in both trees (ab_old/ and this one)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for t in ab_old .; do
  n=$([ $t = . ] && echo new || echo old)
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/dg_$n -o run -- \
      python3 $R/$t/scripts/job_timing.py mul 200 > $R/gpurun_out/dg_$n.log 2>&1 || exit 1
  python3 -c "
import csv,glob
f=glob.glob('$R/gpurun_out/dg_$n/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'k_digits' in r['Name'] or 'gemm16s' in r['Name']: print('$n', r['Name'][:60], r['Calls'], 'avg', round(float(r['AverageNs'])/1e3,2), 'min', round(float(r['MinNs'])/1e3,2))"
done
bash $R/scripts/gpu_ab_trees.sh "mul:300" 3 ab_old . || exit 1
