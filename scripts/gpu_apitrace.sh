#!/bin/bash
# HIP API call statistics of single jobs (host overhead analysis)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/api_${1:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for job in lr msb; do
  timeout -k 10 240 rocprofv3 --hip-trace --stats --output-format csv -d $O/$job -o run -- \
      python3 $R/scripts/prof_job.py --job $job --steps 20 > $O/$job.log 2>&1 || exit $?
done
echo api_ok
