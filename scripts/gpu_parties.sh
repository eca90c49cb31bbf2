#!/bin/bash
# three-party-process transport on the GPU box: its tests, then the bench
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parties.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_parties.log 2>&1
rc=$?; echo pytest_rc=$rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
echo bench_ok
