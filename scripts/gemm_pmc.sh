#!/bin/bash
# one PMC pass over the standalone share GEMM: gemm_pmc.sh <size> <counters>
R=$GRAFT_REPO_ROOT
SZ=$1; CT=$2
cd /tmp && export TMPDIR=/tmp
for v in gemm; do
  O=$R/gpurun_out/pmc_$v
  mkdir -p $O
  timeout -s KILL 120 rocprofv3 --pmc $CT --output-format csv -d $O -o run -- python3 $R/scripts/bench_gemm.py $SZ > $O/log 2>&1 || exit $?
  python3 - $O <<'PY'
import csv, collections, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(float); disp = set(); dur = {}
for r in csv.DictReader(open(f)):
    if "share_gemm" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
n = len(disp); d = sum(dur.values()) / n
print(sys.argv[1].split("/")[-1], "dispatches", n, "avg_ns", round(d), {k: round(v / n) for k, v in agg.items()})
PY
done
