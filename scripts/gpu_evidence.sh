#!/bin/bash
# One GPU call of round evidence, in the driver's order: the whole
# `pytest -m gpu` suite once, smoke(), the default bench line, then the
# rocprofv3 passes (scripts/gpu_profile.sh) unless NOPROF=1.
#   gpurun -- bash scripts/gpu_evidence.sh r06a
R=$GRAFT_REPO_ROOT
TAG=${1:-r06}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
echo bench_ok
[ "${NOPROF:-0}" = 1 ] || bash scripts/gpu_profile.sh $TAG || exit $?
echo evidence_ok
