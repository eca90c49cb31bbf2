#!/bin/bash
# Kernel traces of one job run as three party processes on GPU 0 (the
# north_star layout on one GPU), each party under its own rocprofv3, plus the
# same job co-located in one process, for a side-by-side timeline
# (scripts/party_timeline.py).   prof_parties.sh TAG JOB PARAMS STEPS WARMUP
R=$GRAFT_REPO_ROOT
TAG=$1; JOB=$2; PARAMS=$3; STEPS=${4:-20}; WARM=${5:-20}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
L=pp$$
pids=()
for p in 0 1 2; do
  ABY3_LINK_TIMEOUT_S=60 ABY3_WARMUP_STEPS=$WARM timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/p$p -o run -- python3 $R/tests/party_worker.py $JOB $p $STEPS $L 0 $PARAMS 1 > $O/p$p.json 2> $O/p$p.err &
  pids+=($!)
done
rc=0
for pid in "${pids[@]}"; do wait $pid || rc=$?; done
[ $rc = 0 ] || { tail -5 $O/p*.err; exit $rc; }
python3 $R/scripts/party_timeline.py $O > $O/timeline.txt || exit $?
tail -30 $O/timeline.txt
