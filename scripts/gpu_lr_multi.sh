#!/bin/bash
# several SGD_Logistic iterations per launch: share-exact against one per launch, then A/B
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python -u -c "
import sys; sys.path.insert(0,'.')
from aby3_amd import native as nt
base=[100000,128,256,16,11,0]
ref=None
for k in (1, 8, 3, 64):
    with nt.Session(nt.JOB_LR, base+[k], probe=False) as s:
        s.run(37); d=[s.digest(p) for p in range(3)]; ok=s.check(); info=s.info()
    print('per_launch', k, 'ok', ok, 'fused', info['lr_fused'], d, flush=True)
    assert ok
    if ref is None: ref=d
    assert d==ref, 'digests differ'
print('multi share-exact')
" || exit 1
for i in 1 2; do
  for k in 1 4 16; do ABY3_LR_ITERS_PER_LAUNCH=$k AB_TAG=k$k timeout -k 10 120 python scripts/job_timing.py lr 2000 2>&1 | tail -2 || exit 1; done
done
