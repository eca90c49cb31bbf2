#!/bin/bash
# full GPU test suite, then the bench line without CPU legs
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 --warmup 10 ${BENCH_ARGS} > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_q.json'));e=d.get('extras',{})
print('C2',round(d['ms_per_step'],4),'frac',round(d['roofline']['frac'],3),'C3',round(d['binary']['ms_per_step'],4),'C4',round(e.get('lr_iteration',{}).get('ms_per_iteration',0),4),'C5',round(e.get('merge_sort',{}).get('ms_per_sort',0),2))"
