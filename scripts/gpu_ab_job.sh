#!/bin/bash
# same-box A/B of one job (scripts/job_timing.py) between the baseline tree
# ab_old/ and this tree: gpu_ab_job.sh JOB STEPS [rounds]
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
JOB=$1; ST=${2:-100}; N=${3:-3}
for i in $(seq 1 $N); do
  for t in old new; do
    if [ $t = old ]; then D=ab_old; else D=.; fi
    AB_TAG=$t timeout -k 10 300 python $D/scripts/job_timing.py $JOB $ST || exit 1
  done
done
