#!/bin/bash
# SQ counters of the share GEMM inside the C2 job (each launch alone under the
# PMC pass): where its waves spend their cycles. gemm_sq_pmc.sh TAG
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
    --output-format csv -d $O/pmc_sq -o run -- python3 $R/scripts/prof_job.py --job mul --steps 4 > $O/pmc_sq.log 2>&1 || exit $?
python3 - $O/pmc_sq <<'PY'
import csv, collections, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(float); disp = set()
for r in csv.DictReader(open(f)):
    if "k_share_gemm" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
n = len(disp)
print("dispatches", n, {k: round(v / n) for k, v in sorted(agg.items())})
PY
