#!/bin/bash
# helper rows kept between the two dataset products: LR parity, then A/B
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_protocols.py tests/test_gpu_parties.py tests/test_lr_driver.py -m gpu -k "lr or LR or sgd" > gpurun_out/lr_keep_tests.log 2>&1 \
    || { grep -E "FAIL|Error|error" gpurun_out/lr_keep_tests.log | head -20; tail -5 gpurun_out/lr_keep_tests.log; exit 1; }
tail -1 gpurun_out/lr_keep_tests.log
for i in 1 2 3; do
  for k in 0 1; do ABY3G_LR_KEEP_ROWS=$k AB_TAG=keep$k timeout -k 10 120 python scripts/job_timing.py lr 2000 || exit 1; done
done
