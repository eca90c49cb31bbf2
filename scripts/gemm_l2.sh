#!/bin/bash
# L2 / TA counters of the standalone share GEMM, one PMC pass each
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gl2_${1:-x}
SZ=${2:-4096x4096x4096}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --output-format csv -d $O/p1 -o run -- python3 $R/scripts/bench_gemm.py $SZ > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM --output-format csv -d $O/p2 -o run -- python3 $R/scripts/bench_gemm.py $SZ > $O/p2.log 2>&1
echo counters_rc=$?
