#!/bin/bash
# rocprofv3 kernel trace + stats of the share-conversion jobs (10 steps each)
# and one FETCH_SIZE / WRITE_SIZE pass per job, for profiles/<tag>_conv_*.
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
O=$R/gpurun_out/${TAG}_conv
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for job in a2b bitinj; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$job -o run -- \
      python3 $R/scripts/prof_job.py --job $job --steps 10 > $O/trace_$job.log 2>&1 || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${job}_$c -o run -- \
        python3 $R/scripts/prof_job.py --job $job --steps 4 > $O/pmc_${job}_$c.log 2>&1 || exit $?
  done
done
echo profile_ok
