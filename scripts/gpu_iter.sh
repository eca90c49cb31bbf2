#!/bin/bash
# iteration pass on the GPU box: the GPU tests selected by $1 (pytest -k
# expression; "all" = every GPU test), then the bench line without CPU legs
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
K=${1:-all}
if [ "$K" = "all" ]; then KARG=(); else KARG=(-k "$K"); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread "${KARG[@]}" > gpurun_out/pytest_iter.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_iter.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error|Timeout" gpurun_out/pytest_iter.log | head -30; exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 50 --warmup 10 ${BENCH_ARGS} > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err || { tail -20 gpurun_out/bench_iter.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench_iter.json'));e=d.get('extras',{})
print('C2',round(d['ms_per_step'],4),'frac',round(d['roofline']['frac'],3),'lcf',round(d['local_compute_fraction'],3),'C3',round(d['binary']['ms_per_step'],4),'C3lcf',round(d['binary']['local_compute']['local_compute_fraction'],3),'C4',round(e.get('lr_iteration',{}).get('ms_per_iteration',0),4),'C5',round(e.get('merge_sort',{}).get('ms_per_sort',0),2),'a2b',round(e.get('a2b',{}).get('ms_per_conversion',0),3))"
