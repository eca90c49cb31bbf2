#!/bin/bash
# binary engine fused forms: parity with them on, then the C3 A/B and a trace
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ABY3_FUSE_INPUTS=1 ABY3_MERGE_LEVELS=1 timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_gpu_protocols.py tests/test_cpp.py::test_binary_protocols_gpu -m gpu -k "cipher_gt or session_jobs or binary or circuit" \
    > gpurun_out/r04b_tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r04b_tests.log | head -20; tail -5 gpurun_out/r04b_tests.log; exit 1; }
tail -1 gpurun_out/r04b_tests.log
for i in 1 2; do
  for fmo in 000 100 101 110 010; do
    ABY3_FUSE_INPUTS=${fmo:0:1} ABY3_MERGE_LEVELS=${fmo:1:1} ABY3_FUSE_OUTPUT=${fmo:2:1} AB_TAG=in_merge_out$fmo timeout -k 10 120 python scripts/job_timing.py msb 300 || exit 1
  done
done
ABY3_FUSE_INPUTS=1 ABY3_MERGE_LEVELS=1 KT_STEPS=20 bash scripts/gpu_ktrace.sh r04 msb || exit 1
python3 scripts/timeline.py $(ls gpurun_out/kt_r04/msb/*kernel_trace.csv | head -1) 0.5 110 > gpurun_out/c3_timeline.txt
tail -3 gpurun_out/c3_timeline.txt
