#!/bin/bash
# Baseline of the latency-bound jobs: bench line (no CPU legs), then per job a
# HIP API trace and a kernel trace of 20 steps (scripts/prof_job.py).
#   usage: gpu_jobprof.sh TAG [jobs...]   (default jobs: lr msb)
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
shift
JOBS=${@:-lr msb}
O=$R/gpurun_out/jp_$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 --warmup 10 > $O/bench.json 2> $O/bench.err || exit $?
echo bench_ok
cd /tmp && export TMPDIR=/tmp
for job in $JOBS; do
  timeout -k 10 200 rocprofv3 --hip-trace --stats --output-format csv -d $O/api_$job -o run -- \
      python3 $R/scripts/prof_job.py --job $job --steps 20 > $O/api_$job.log 2>&1 || exit $?
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$job -o run -- \
      python3 $R/scripts/prof_job.py --job $job --steps 20 > $O/k_$job.log 2>&1 || exit $?
  echo ${job}_ok
done
