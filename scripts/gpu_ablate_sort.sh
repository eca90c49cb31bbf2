#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do
AB_TAG=base timeout -k 10 200 python scripts/job_timing.py sort 3
ABY3_DEBUG_NOSCATTER=1 AB_TAG=noscatter timeout -k 10 200 python scripts/job_timing.py sort 3
ABY3_DEBUG_NOGATHER=1 AB_TAG=nogather timeout -k 10 200 python scripts/job_timing.py sort 3
done
exit 0
