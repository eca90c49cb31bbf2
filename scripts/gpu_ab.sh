#!/bin/bash
# quick A/B pass on the GPU box: the GEMM / epilogue parity tests, then the
# C2 bench line under each variant given as "NAME=VALUE ..." arguments
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_protocols.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread -k "mul or gemm or trunc or session" > gpurun_out/pytest_ab.log 2>&1 || exit $?
echo tests_ok
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 120 python bench.py --no-extras --no-binary --no-cpu-baseline --steps 100 > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || exit $?
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));print(round(d['ms_per_step'],4), d['kernel_ms_per_step'], round(d['roofline']['frac'],3))")"
done
