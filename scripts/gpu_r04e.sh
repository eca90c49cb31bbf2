#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for i in 1 2 3; do
  for j in mul mul2; do AB_TAG=$j timeout -k 10 120 python scripts/job_timing.py $j 300 || exit 1; done
done
timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'.')
from aby3_amd import native as nt
d=[]
for p in ([1024,1024,1024,16,1],[1024,1024,1024,16,1,2]):
    with nt.Session(nt.JOB_MUL_TRUNC, p, probe=False) as s:
        s.run(7); d.append([s.digest(i) for i in range(3)]); assert s.check()
print('digests equal', d[0]==d[1], d)
" || exit 1
KT_STEPS=40 bash scripts/gpu_ktrace.sh r04e mul || exit 1
python3 scripts/timeline.py $(find gpurun_out/kt_r04e/mul -name "*kernel_trace.csv" | head -1) 0.6 70 > gpurun_out/c2_timeline.txt
