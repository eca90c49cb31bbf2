#!/bin/bash
# three party processes of one job on GPU 0 for each tree given, alternating:
# parties_ab.sh JOB STEPS PARAMS ROUNDS tree...
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
JOB=$1; STEPS=$2; PARAMS=$3; N=$4; shift 4
for i in $(seq 1 $N); do
  for tree in "$@"; do
    pids=""
    for p in 0 1 2; do
      ABY3_LINK_TIMEOUT_S=60 ABY3_WARMUP_STEPS=50 timeout -k 5 120 python $tree/$( [ -e $tree/scripts/party_worker.py ] && echo scripts || echo tests)/party_worker.py $JOB $p $STEPS ab$$.$i.${tree//\//_} 0 $PARAMS \
          > gpurun_out/pab.$p.out 2> gpurun_out/pab.$p.err &
      pids="$pids $!"
    done
    wait $pids || { cat gpurun_out/pab.*.err | tail -20; exit 1; }
    echo "$tree $JOB $(python3 -c "import json,sys; print(max(json.loads(open('gpurun_out/pab.%d.out'%p).read().strip().splitlines()[-1])['ms_per_step'] for p in range(3)))")"
  done
done
