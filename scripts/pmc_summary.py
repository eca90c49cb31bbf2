"""Summarises rocprofv3 CSV output (kernel stats and PMC passes) into
profiles/pmc_<tag>.json for bench.py's `traffic` fields.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: rocprofv3 reports
both in KiB, and on gfx950 FETCH_SIZE counts half the bytes of wide coalesced
streaming reads (MI355X_MICROARCH.md §HBM), hence the factor 2 on the read
side. All kernels here read with 16-byte-per-lane loads.

usage: pmc_summary.py --fetch DIR --write DIR --steps S --job mul|msb --out FILE
       pmc_summary.py --recompute FILE --steps S   (re-derive bin_gates from
                                                    the file's kernel table)
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


# Kernels that run the binary engine's gate levels: every launch form of a
# level (k_bin_level, the fused first level k_bin_level_in, the merged light
# levels k_bin_levels, the level with its output read-out k_bin_level_out) and
# the older split forms. The binary roofline's traffic is their sum; the CPU
# contract test (tests/test_bench_contract.py) checks that every such kernel in
# the committed kernel stats is matched here.
LEVEL_PREFIXES = ("k_bin_level", "k_bin_gates", "k_bin_unpack")


def is_level_kernel(name):
    return name.startswith(LEVEL_PREFIXES)


def bin_level_bytes(kernels):
    return sum(v["read_bytes"] + v["write_bytes"] for k, v in kernels.items() if is_level_kernel(k))


def per_kernel(d, counter):
    tot = collections.defaultdict(float)
    n = collections.defaultdict(int)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            m = re.search(r"\b(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:60]
            tot[k] += float(r["Counter_Value"])
            n[k] += 1
    return tot, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--job", choices=["mul", "msb"])
    ap.add_argument("--out")
    ap.add_argument("--recompute")
    a = ap.parse_args()
    if a.recompute:
        out = json.load(open(a.recompute))
        out["bin_gates"]["hbm_bytes_per_step_per_party"] = bin_level_bytes(out["kernels"]["msb"]) / (3 * a.steps)
        json.dump(out, open(a.recompute, "w"), indent=1)
        print(out["bin_gates"])
        return
    ft, fn = per_kernel(a.fetch, "FETCH_SIZE")
    wt, wn = per_kernel(a.write, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(ft) | set(wt)):
        launches = max(fn.get(k, 0), wn.get(k, 0))
        rd = 2 * ft.get(k, 0.0) * 1024
        wr = wt.get(k, 0.0) * 1024
        kernels[k] = dict(launches=launches, read_bytes=rd, write_bytes=wr,
                          hbm_bytes_per_launch=(rd + wr) / max(launches, 1))
    out = json.load(open(a.out)) if os.path.exists(a.out) else {}
    out.setdefault("note", "HBM bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 per rocprofv3 --pmc passes; "
                           "gfx950 FETCH_SIZE read-side correction x2")
    party_steps = 3 * a.steps
    if a.job == "mul":
        g = next((v for k, v in kernels.items() if k.startswith("k_share_gemm")), {})
        out["share_gemm"] = dict(config={"m": 1024, "k": 1024, "n": 1024},
                                 hbm_bytes_per_launch=g.get("hbm_bytes_per_launch"), launches=g.get("launches"))
    else:
        tot = bin_level_bytes(kernels)
        out["bin_gates"] = dict(config={"rows": 1 << 20}, hbm_bytes_per_step_per_party=tot / party_steps,
                                hbm_bytes_per_launch=None)
    out.setdefault("kernels", {})[a.job] = kernels
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main()
