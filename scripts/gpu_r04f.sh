#!/bin/bash
# C3 kernel trace in the default configuration + per-kernel sums per step
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
KT_STEPS=30 bash scripts/gpu_ktrace.sh r04f msb || exit 1
F=$(find gpurun_out/kt_r04f/msb -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $F 0.6 120 > gpurun_out/c3_timeline_def.txt
