#!/bin/bash
# kernel trace (concurrent, as in the bench) of single jobs: gpu_ktrace.sh TAG jobs...
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
shift
O=$R/gpurun_out/kt_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for job in ${@:-mul msb}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$job -o run -- \
      python3 $R/scripts/prof_job.py --job $job --steps ${KT_STEPS:-20} > $O/$job.log 2>&1 || exit $?
  echo ${job}_ok
done
