#!/bin/bash
# MFMA utilisation of the share GEMM in the C2 job (co-located plan: 128
# workgroups per launch; the PMC pass serialises kernels, so each launch runs
# alone): SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE (the clock) per dispatch.
# usage: gemm_mfma_pmc.sh TAG   -> gpurun_out/TAG/pmc_mfma + mfma_summary.json
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d $O/pmc_mfma -o run -- python3 $R/scripts/prof_job.py --job mul --steps 4 > $O/pmc_mfma.log 2>&1 || exit $?
python3 $R/scripts/mfma_summary.py $O/pmc_mfma $O/mfma_summary.json
