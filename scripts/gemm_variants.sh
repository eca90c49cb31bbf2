#!/bin/bash
# A/B of the share-GEMM kernel variants (standalone, one stream)
# usage: gemm_variants.sh [variants...] (default: b c a d)
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
VS=${@:-b c a d}
for v in $VS; do
  echo "variant $v"
  ABY3G_GEMM_VARIANT=$v timeout -k 10 120 python $GRAFT_REPO_ROOT/scripts/bench_gemm.py 1024x1024x1024 4096x4096x4096 || exit $?
done
