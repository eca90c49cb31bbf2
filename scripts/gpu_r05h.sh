#!/bin/bash
# round-5 A/B: the fused merge-round forms (slot counts) and the LR solo levels
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
O=gpurun_out/ab_r05h.log
for i in 1 2; do
  AB_TAG=old timeout -k 10 300 python ab_old/scripts/job_timing.py sort 3 >> $O || exit 1
  AB_TAG=old timeout -k 10 300 python ab_old/scripts/job_timing.py lr 2000 >> $O || exit 1
  for v in "X=0" "ABY3G_TMP_OUT8=1" "ABY3G_TMP_IN8=1" "ABY3G_TMP_OUT8=1 ABY3G_TMP_IN8=1" "ABY3_FUSE_INPUTS=0"; do
    env $v AB_TAG="$v" timeout -k 10 300 python scripts/job_timing.py sort 3 >> $O || exit 1
  done
  AB_TAG=new timeout -k 10 300 python scripts/job_timing.py lr 2000 >> $O || exit 1
  AB_TAG=new timeout -k 10 300 python scripts/job_timing.py msb 300 >> $O || exit 1
done
timeout -k 10 120 python -u -m pytest tests/test_golden.py -x -v -s -p no:cacheprovider --timeout 100 --timeout-method thread -k merge_gpu > gpurun_out/hd_r05.log 2>&1
