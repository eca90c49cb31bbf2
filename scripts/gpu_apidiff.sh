#!/bin/bash
# steady-state HIP API calls per step of one job: hip-trace stats at two step counts
R=$GRAFT_REPO_ROOT
J=${1:-lr}
O=$R/gpurun_out/apid_$J
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in 10 60; do
  timeout -k 10 200 rocprofv3 --hip-trace --stats --output-format csv -d $O/s$n -o run -- \
      python3 $R/scripts/prof_job.py --job $J --steps $n > $O/s$n.log 2>&1 || exit $?
done
echo ok
