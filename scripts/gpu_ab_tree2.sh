#!/bin/bash
# same-box A/B of two trees: ab_old/ (an earlier commit, built in place) and
# the current tree, alternating: gpu_ab_tree2.sh "job:steps ..." [rounds]
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
JOBS=$1; N=${2:-2}
for i in $(seq 1 $N); do
  for tree in ab_old .; do
    for js in $JOBS; do
      job=${js%%:*}; st=${js##*:}
      AB_TAG=$tree timeout -k 10 300 python $tree/scripts/job_timing.py $job $st || exit 1
    done
  done
done
