#!/bin/bash
# host API + kernel trace of one job, to read launch-to-start delays (is the
# host or the device on the critical path?): gpu_hostdev.sh TAG job steps
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/hd_${1:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/${2:-msb} -o run -- \
    python3 $R/scripts/prof_job.py --job ${2:-msb} --steps ${3:-20} > $O/${2:-msb}.log 2>&1 || exit $?
echo hd_ok
