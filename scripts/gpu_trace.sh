#!/bin/bash
# kernel-trace timelines of single jobs (mul, lr), for reading critical paths
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trace_${1:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for job in mul lr msb; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/$job -o run -- \
      python3 $R/scripts/prof_job.py --job $job --steps 20 > $O/$job.log 2>&1 || exit $?
done
echo trace_ok
