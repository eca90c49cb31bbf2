#!/bin/bash
# C4 (one SGD_Logistic iteration) with each party in its own process on GPU 0
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
L=lrp$$
for p in 0 1 2; do
  ABY3_LINK_TIMEOUT_S=120 timeout -k 10 200 python tests/party_worker.py 3 $p ${1:-100} $L 0 1000000,128,256,16,11 > gpurun_out/lrp_$p.json 2> gpurun_out/lrp_$p.err &
done
wait
cat gpurun_out/lrp_*.json
