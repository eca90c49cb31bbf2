#!/bin/bash
# LR helper messages as granules: the LR parity tests, then a same-box C4 A/B
# against ab_old/ (the tree before), then the new tree's phase profile
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_cpp.py::test_lr_iteration_both_forms_gpu tests/test_lr_driver.py tests/test_gpu_parties.py -k "lr or LR or 3-" \
    > gpurun_out/lr_tests.log 2>&1 || { tail -30 gpurun_out/lr_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 gpurun_out/lr_tests.log
bash scripts/gpu_ab_trees.sh "lr:1000" 4 ab_old . || exit 1
timeout -k 10 120 ./scripts/lr_phases 1000000 300 > gpurun_out/lr_phases.txt 2>&1 || { cat gpurun_out/lr_phases.txt; exit 1; }
head -8 gpurun_out/lr_phases.txt
