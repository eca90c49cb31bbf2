#!/bin/bash
# three party processes of one job on GPU 0 per environment setting, alternating:
# parties_ab_env.sh JOB STEPS PARAMS ROUNDS "VAR=v ..." ...
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
JOB=$1; STEPS=$2; PARAMS=$3; N=$4; shift 4
for i in $(seq 1 $N); do
  for setting in "$@"; do
    pids=""
    tag=abe$$.$i.$RANDOM
    for p in 0 1 2; do
      env $setting ABY3_LINK_TIMEOUT_S=60 ABY3_WARMUP_STEPS=50 timeout -k 5 120 python tests/party_worker.py $JOB $p $STEPS $tag 0 $PARAMS \
          > gpurun_out/pab.$p.out 2> gpurun_out/pab.$p.err &
      pids="$pids $!"
    done
    wait $pids || { cat gpurun_out/pab.*.err | tail -20; exit 1; }
    echo "$setting $JOB $(python3 -c "import json,sys; print(max(json.loads(open('gpurun_out/pab.%d.out'%p).read().strip().splitlines()[-1])['ms_per_step'] for p in range(3)))")"
  done
done
