#!/bin/bash
# the LR parity tests (C++ both forms vs oracle, Python vs oracle/fixture), the
# fused iteration's phase profile and the C4 job timing
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_cpp.py::test_lr_iteration_both_forms_gpu tests/test_lr_driver.py tests/test_gpu_parties.py -k "lr or LR or 3-" \
    > gpurun_out/lr_tests.log 2>&1 || { tail -30 gpurun_out/lr_tests.log; exit 1; }
tail -1 gpurun_out/lr_tests.log
timeout -k 10 120 ./scripts/lr_phases 1000000 300 > gpurun_out/lr_phases.txt 2>&1 || { cat gpurun_out/lr_phases.txt; exit 1; }
cat gpurun_out/lr_phases.txt
timeout -k 10 120 python scripts/job_timing.py lr 1000
KT_STEPS=20 bash scripts/gpu_ktrace.sh r04 msb || exit 1
python3 scripts/timeline.py $(ls gpurun_out/kt_r04/msb/*kernel_trace.csv | head -1) 0.5 110 > gpurun_out/c3_timeline.txt
tail -3 gpurun_out/c3_timeline.txt
