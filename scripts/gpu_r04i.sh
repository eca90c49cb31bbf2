#!/bin/bash
# host launch time vs device start of the mask draws (HIP API + kernel trace)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/hk_r04i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O -o run -- \
    python3 $R/scripts/prof_job.py --job msb --steps 30 > $O/run.log 2>&1 || exit $?
echo ok
