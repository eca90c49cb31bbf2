#!/bin/bash
# 32-column digit workgroups: GEMM parity, then C2 A/B
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_kernels.py tests/test_gpu_protocols.py -m gpu -k "mul or digit or gemm or session_jobs" > gpurun_out/digits_tests.log 2>&1 \
    || { grep -E "FAIL|Error|error" gpurun_out/digits_tests.log | head -20; tail -5 gpurun_out/digits_tests.log; exit 1; }
tail -1 gpurun_out/digits_tests.log
for i in 1 2 3; do
  for c in 64 32; do ABY3G_DIGIT_COLS=$c AB_TAG=cols$c timeout -k 10 120 python scripts/job_timing.py mul 300 || exit 1; done
done
