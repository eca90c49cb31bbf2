#!/bin/bash
# kernel durations (rocprofv3) of the standalone transposes at several sizes
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for rows in 262144 1048576 8388608; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/b2w_$rows -o run -- python3 $R/scripts/bench_binary.py $rows > $R/gpurun_out/b2w_$rows.log 2>&1 || exit $?
done
echo done
