#!/bin/bash
# same-box A/B of trees built in place (ab_old/, ab_v1/, ... and the current
# tree "."), alternating: gpu_ab_trees.sh "job:steps ..." rounds tree...
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
JOBS=$1; N=$2; shift 2
for i in $(seq 1 $N); do
  for tree in "$@"; do
    for js in $JOBS; do
      job=${js%%:*}; st=${js##*:}
      AB_TAG=$tree timeout -k 10 300 python $tree/scripts/job_timing.py $job $st || exit 1
    done
  done
done
