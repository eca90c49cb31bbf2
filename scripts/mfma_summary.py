"""Summarises the MFMA PMC pass of scripts/gemm_mfma_pmc.sh: per share-GEMM
dispatch the MFMA-busy cycles, the effective clock (GRBM_GUI_ACTIVE / 8 XCDs
/ wall time, MI355X_MICROARCH.md 'DVFS give-back') and the busy fraction of
the SIMDs the launch occupies (128 workgroups = 128 CUs x 4 SIMDs), against
the instruction count the kernel issues (5.24 M v_mfma_i32_16x16x64_i8 at
1024^3, 16 cycles each).

usage: mfma_summary.py PMC_DIR OUT_JSON"""
import collections
import csv
import glob
import json
import sys

d, out = sys.argv[1], sys.argv[2]
f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
per = collections.defaultdict(dict)
dur = {}
for r in csv.DictReader(open(f)):
    if "k_share_gemm" not in r["Kernel_Name"]:
        continue
    k = r["Dispatch_Id"]
    per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    dur[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
n = len(per)
avg = {c: sum(v[c] for v in per.values()) / n for c in next(iter(per.values()))}
ns = sum(dur.values()) / n
mfmas = 128 * 8 * 64 * 80  # workgroups x waves x K' stages x MFMAs per wave and stage (1024^3)
cycles16 = mfmas * 16
clock = avg["GRBM_GUI_ACTIVE"] / 8 / (ns * 1e-9)
simds = 128 * 4
res = dict(
    dispatches=n, avg_ns=ns, counters=avg, mfma_instructions=mfmas, mfma_cycles_if_16_each=cycles16,
    mfma_busy_over_issued_cycles=avg["SQ_VALU_MFMA_BUSY_CYCLES"] / cycles16,
    effective_clock_ghz=clock / 1e9,
    mfma_busy_frac_of_occupied_simds=avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (simds * avg["GRBM_GUI_ACTIVE"] / 8),
    note="one launch alone (the PMC pass serialises kernels); 128 workgroups on 128 CUs",
)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
