#!/bin/bash
# same-box A/B of one environment variable: gpu_ab_env.sh VAR "v1 v2 ..." "job:steps ..." [rounds]
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
VAR=$1; VALS=$2; JOBS=$3; N=${4:-2}
for i in $(seq 1 $N); do
  for v in $VALS; do
    for js in $JOBS; do
      job=${js%%:*}; st=${js##*:}
      env $VAR=$v AB_TAG="$VAR=$v" timeout -k 10 300 python scripts/job_timing.py $job $st || exit 1
    done
  done
done
