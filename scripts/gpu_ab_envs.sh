#!/bin/bash
# same-box A/B of environment settings: gpu_ab_envs.sh "job:steps ..." rounds "VAR=v ..." "VAR=v ..." ...
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
JOBS=$1; N=$2; shift 2
for i in $(seq 1 $N); do
  for setting in "$@"; do
    for js in $JOBS; do
      job=${js%%:*}; st=${js##*:}
      env $setting AB_TAG="$setting" timeout -k 10 300 python scripts/job_timing.py $job $st || exit 1
    done
  done
done
