#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do
AB_TAG=base timeout -k 10 120 python scripts/job_timing.py msb 300
ABY3_DEBUG_NODRAW=1 AB_TAG=nodraw timeout -k 10 120 python scripts/job_timing.py msb 300
done
ABY3_DEBUG_NODRAW=1 AB_TAG=nodraw timeout -k 10 200 python scripts/job_timing.py sort 3
AB_TAG=base timeout -k 10 200 python scripts/job_timing.py sort 3
timeout -k 10 300 python -c "
import sys, os, json; sys.argv=['x']; sys.path.insert(0,'.')
import bench
from aby3_amd import native as nt
for pd in ('0','1'):
    os.environ['ABY3_PARTY_DRAW_STREAM']=pd
    ms, outs = bench.party_job(nt.JOB_MSB, [1<<20], 30, warmup=50)
    print(json.dumps(dict(job='msb_party', draw_stream=pd, party_ms=round(ms, 4))))
"
exit 0
