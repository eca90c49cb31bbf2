#!/bin/bash
# Standalone kernel durations in situ: kernel trace of single jobs with every
# kernel serialised (AMD_SERIALIZE_KERNEL=3; the channels then use events).
#   usage: gpu_serial.sh TAG [jobs...]   (default jobs: msb mul)
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
shift
JOBS=${@:-msb mul}
O=$R/gpurun_out/ser_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export AMD_SERIALIZE_KERNEL=3
for job in $JOBS; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$job -o run -- \
      python3 $R/scripts/prof_job.py --job $job --steps 10 > $O/k_$job.log 2>&1 || exit $?
  echo ${job}_ok
done
