#!/bin/bash
# round-end evidence in one call: pytest -m gpu, smoke, the default bench
# line, the rocprofv3 kernel-trace / PMC passes (scripts/gpu_profile.sh) and
# the C4 API-call difference (scripts/gpu_apidiff.sh lr)
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
echo bench_ok
bash scripts/gpu_profile.sh $TAG || exit $?
bash scripts/gpu_apidiff.sh lr || exit $?
python3 scripts/apidiff_summary.py gpurun_out/apid_lr/s10 gpurun_out/apid_lr/s60 10 60 \
    "C4 (fused LR iteration, 100000x128 dataset, batch 256): steady-state HIP API calls per party per iteration" \
    > gpurun_out/$TAG/c4_api_calls.txt || exit $?
echo round_end_ok
