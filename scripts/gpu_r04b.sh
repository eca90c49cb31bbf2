#!/bin/bash
# LR drawn-ahead randomness + fused first binary level: parity tests, LR
# phases, C3/C4/C5 job timings A/B (ABY3_FUSE_INPUTS), C3 kernel trace
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_cpp.py tests/test_lr_driver.py tests/test_gpu_protocols.py -m gpu \
    > gpurun_out/r04b_tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r04b_tests.log | head -20; tail -5 gpurun_out/r04b_tests.log; exit 1; }
tail -1 gpurun_out/r04b_tests.log
timeout -k 10 120 ./scripts/lr_phases 1000000 300 > gpurun_out/lr_phases.txt 2>&1 || { cat gpurun_out/lr_phases.txt; exit 1; }
cat gpurun_out/lr_phases.txt
for i in 1 2; do
  for fm in 00 10 11; do
    ABY3_FUSE_INPUTS=${fm:0:1} ABY3_MERGE_LEVELS=${fm:1:1} AB_TAG=fuse_merge$fm timeout -k 10 120 python scripts/job_timing.py msb 200 || exit 1
  done
done
timeout -k 10 120 python scripts/job_timing.py lr 2000 || exit 1
ABY3_FUSE_INPUTS=1 AB_TAG=fuse1 timeout -k 10 200 python scripts/job_timing.py sort 3 || exit 1
KT_STEPS=20 bash scripts/gpu_ktrace.sh r04 msb || exit 1
python3 scripts/timeline.py $(ls gpurun_out/kt_r04/msb/*kernel_trace.csv | head -1) 0.5 110 > gpurun_out/c3_timeline.txt
tail -3 gpurun_out/c3_timeline.txt
