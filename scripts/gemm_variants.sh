#!/bin/bash
# A/B of the share-GEMM kernel variants (standalone, one stream)
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
for v in b c a d; do
  echo "variant $v"
  ABY3G_GEMM_VARIANT=$v timeout -k 10 120 python $GRAFT_REPO_ROOT/scripts/bench_gemm.py 1024x1024x1024 4096x4096x4096 || exit $?
done
