#!/bin/bash
# digit split with 16-byte A loads: the share-GEMM parity tests, then a
# same-box C2 A/B against ab_old/ (the tree before)
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -m gpu \
    tests -k "mul_local or mul_trunc or digit or gemm" > gpurun_out/digits_tests.log 2>&1 || { tail -30 gpurun_out/digits_tests.log; exit 1; }
tail -1 gpurun_out/digits_tests.log
bash scripts/gpu_ab_trees.sh "mul:300" 4 ab_old . || exit 1
