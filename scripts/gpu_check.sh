#!/bin/bash
# one GPU validation pass: tests, smoke, bench, kernel-trace profile
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 30 --warmup 10 --no-extras --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1
echo prof_rc=$?
