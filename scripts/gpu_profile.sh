#!/bin/bash
# rocprofv3 passes for the round's profiles/: kernel trace + stats of the
# bench, then separate FETCH_SIZE / WRITE_SIZE passes of the two jobs.
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
# GEMMs take turns in this run, so every launch span is the kernel's own (bench.py roofline pass)
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --steps 30 --warmup 10 --no-extras --no-cpu-baseline --gemm-turns > $O/trace.log 2>&1 || exit $?
for job in mul msb; do
  for c in FETCH_SIZE WRITE_SIZE; do
    # counter passes serialise kernels: the channels see ROCPROF_COUNTER_COLLECTION and use events
    timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${job}_$c -o run -- \
        python3 $R/scripts/prof_job.py --job $job --steps 4 > $O/pmc_${job}_$c.log 2>&1 || exit $?
  done
  python3 $R/scripts/pmc_summary.py --fetch $O/pmc_${job}_FETCH_SIZE --write $O/pmc_${job}_WRITE_SIZE \
      --steps 4 --job $job --out $O/pmc_$TAG.json > $O/pmc_summary_$job.log 2>&1 || exit $?
done
echo profile_ok
