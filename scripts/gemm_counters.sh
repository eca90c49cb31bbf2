#!/bin/bash
# SQ counters of the standalone share GEMM (1024^3), one PMC pass
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gc_${1:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $O/p1 -o run -- python3 $R/scripts/bench_gemm.py 1024x1024x1024 > $O/p1.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL TA_BUSY_avr --output-format csv -d $O/p2 -o run -- python3 $R/scripts/bench_gemm.py 1024x1024x1024 > $O/p2.log 2>&1
echo counters_rc=$?
