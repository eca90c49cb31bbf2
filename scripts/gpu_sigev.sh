#!/bin/bash
# same-device message signalling: signal word (stream write/wait) vs event record/wait
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ABY3_SIGNAL_EVENTS=1 timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_protocols.py -m gpu -k "session_jobs or circuit or cipher" > gpurun_out/sigev_tests.log 2>&1 \
    || { grep -E "FAIL|Error|error" gpurun_out/sigev_tests.log | head -20; tail -5 gpurun_out/sigev_tests.log; exit 1; }
tail -1 gpurun_out/sigev_tests.log
for i in 1 2; do
  for e in 0 1; do
    ABY3_SIGNAL_EVENTS=$e AB_TAG=ev$e timeout -k 10 120 python scripts/job_timing.py msb 300 || exit 1
    ABY3_SIGNAL_EVENTS=$e AB_TAG=ev$e timeout -k 10 120 python scripts/job_timing.py mul 300 || exit 1
  done
done
for e in 0 1; do ABY3_SIGNAL_EVENTS=$e AB_TAG=ev$e timeout -k 10 200 python scripts/job_timing.py sort 3 || exit 1; done
