#!/bin/bash
# next batch's rows touched into L2 by the helpers: LR parity, then A/B
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_protocols.py tests/test_gpu_parties.py tests/test_lr_driver.py -m gpu -k "lr or LR or sgd" > gpurun_out/lr_pf_tests.log 2>&1 \
    || { grep -E "FAIL|Error|error" gpurun_out/lr_pf_tests.log | head -20; tail -5 gpurun_out/lr_pf_tests.log; exit 1; }
tail -1 gpurun_out/lr_pf_tests.log
for i in 1 2 3; do
  for k in 0 1; do ABY3_LR_PREFETCH=$k AB_TAG=pf$k timeout -k 10 120 python scripts/job_timing.py lr 2000 || exit 1; done
done
