#!/bin/bash
# pytest -m gpu (the whole suite), then the default bench line
R=$GRAFT_REPO_ROOT
TAG=${1:-r04}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?
tail -1 gpurun_out/$TAG/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error|Timeout" gpurun_out/$TAG/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/$TAG/bench.json'));e=d.get('extras',{})
print('C2',round(d['ms_per_step'],4),'frac',round(d['roofline']['frac'],3),'C3',round(d['binary']['ms_per_step'],4),'C4',round(e.get('lr_iteration',{}).get('ms_per_iteration',0),4),'epoch it/s',round(e.get('lr_epoch',{}).get('iterations_per_s',0)),'C5',round(e.get('merge_sort',{}).get('ms_per_sort',0),2))
print('pp',json.dumps({k:v for k,v in e.get('party_processes',{}).items() if not isinstance(v,dict)}))"
