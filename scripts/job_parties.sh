#!/bin/bash
# one job with each party in its own process on GPU 0:
#   job_parties.sh JOB STEPS PARAMS [LAYOUT]   (LAYOUT: 1 one GPU with arenas, 2 the cross-GPU branches)
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
L=jp$$
LAYOUT=${4:-1}
pids=()
for p in 0 1 2; do
  ABY3_LINK_TIMEOUT_S=120 timeout -k 10 200 python tests/party_worker.py $1 $p $2 $L 0 $3 $LAYOUT > gpurun_out/jp_$p.json 2> gpurun_out/jp_$p.err &
  pids+=($!)
done
rc=0
for pid in "${pids[@]}"; do wait $pid || rc=$?; done
[ $rc = 0 ] || { tail -3 gpurun_out/jp_*.err; exit $rc; }
python3 -c "
import json
r=[json.loads(open(f'gpurun_out/jp_{p}.json').read().strip().splitlines()[-1]) for p in range(3)]
print('job $1 layout $LAYOUT', 'ok', all(x['ok'] for x in r), 'ms_per_step', round(max(x['ms_per_step'] for x in r),4))"
