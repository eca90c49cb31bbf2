#!/bin/bash
# round-end evidence: pytest -m gpu, smoke, default bench line, then the
# rocprofv3 kernel-trace and PMC passes (scripts/gpu_profile.sh TAG)
R=$GRAFT_REPO_ROOT
TAG=${1:-r02}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
echo bench_ok
bash scripts/gpu_profile.sh $TAG
