#!/bin/bash
# round-4 final evidence on the final tree: pytest -m gpu, smoke, the
# driver's bench command and the default one, kernel trace + PMC passes
R=$GRAFT_REPO_ROOT
TAG=${1:-r04c}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/$TAG/pytest_gpu.log | head -20; tail -3 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_driver.json 2> gpurun_out/$TAG/bench_driver.err || exit $?
timeout -k 10 400 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
echo bench_ok
bash scripts/gpu_profile.sh $TAG || exit $?
echo final_ok
