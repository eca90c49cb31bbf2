#!/bin/bash
# binary fused forms + process-layout arenas: parity, then C3 A/B and the party-process timings
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_gpu_parties.py tests/test_gpu_protocols.py -m gpu -k "cipher_gt or session_jobs or circuit or processes or lagging" \
    > gpurun_out/r04c_tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/r04c_tests.log | head -20; tail -5 gpurun_out/r04c_tests.log; exit 1; }
tail -1 gpurun_out/r04c_tests.log
for i in 1 2; do
  for fmo in 000 100 110; do
    ABY3_FUSE_INPUTS=${fmo:0:1} ABY3_MERGE_LEVELS=${fmo:1:1} ABY3_FUSE_OUTPUT=${fmo:2:1} AB_TAG=in_merge_out$fmo timeout -k 10 120 python scripts/job_timing.py msb 300 || exit 1
  done
done
timeout -k 10 300 python -c "
import sys, json; sys.argv=['x']; sys.path.insert(0,'.')
import bench
from aby3_amd import native as nt
for job, params, steps, warm in ((nt.JOB_MSB, [1<<20], 30, 50), (nt.JOB_MUL_TRUNC, [1024,1024,1024,16,1], 30, 100), (nt.JOB_LR, [1000000,128,256,16,11], 300, 1000)):
    ms, outs = bench.party_job(job, params, steps, warmup=warm)
    print(json.dumps(dict(job=job, party_ms=round(ms, 4))))
" || exit 1
# share GEMM with A's digit split inside (k_share_gemm16r): parity, then A/B on C2
ABY3G_GEMM_RAWA=1 timeout -k 10 200 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    tests/test_gpu_kernels.py -m gpu -k "mul_local or mul_trunc_local or digit_extremes or mul_sub" > gpurun_out/r04c_rawa.log 2>&1 \
    || { tail -30 gpurun_out/r04c_rawa.log; exit 1; }
tail -1 gpurun_out/r04c_rawa.log
for i in 1 2 3; do
  for r in 0 1; do ABY3G_GEMM_RAWA=$r AB_TAG=rawa$r timeout -k 10 120 python scripts/job_timing.py mul 200 || exit 1; done
done
