#!/bin/bash
# three party processes of one job on GPU 0, each one's stderr kept:
# parties_dbg.sh JOB STEPS PARAMS LAYOUT TAG
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/pdbg
JOB=$1; STEPS=$2; PARAMS=$3; LAYOUT=$4; TAG=$5
for p in 0 1 2; do
  ABY3_LINK_TIMEOUT_S=${LT:-30} timeout -k 5 90 python tests/party_worker.py $JOB $p $STEPS dbg$$.$TAG 0 $PARAMS $LAYOUT \
      > gpurun_out/pdbg/$TAG.p$p.out 2> gpurun_out/pdbg/$TAG.p$p.err &
done
wait
for p in 0 1 2; do echo "== $TAG party $p"; tail -c 600 gpurun_out/pdbg/$TAG.p$p.err; cat gpurun_out/pdbg/$TAG.p$p.out; done
