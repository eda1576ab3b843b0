#!/usr/bin/env python3
"""Per-launch instruction census of the last bench forward from tools/pmc_forward_insts.sh.

Counts are per launch (SQ_INSTS_* count wave-instructions). VALU excludes nothing: on gfx950
SQ_INSTS_VALU includes the MFMA issues, so 'valu_nonmfma' = VALU - MFMA."""
import csv, collections, json, os, re, sys

base = sys.argv[1]
rows = collections.OrderedDict()
for r in csv.DictReader(open(os.path.join(base, "p1", "run_counter_collection.csv"))):
    d = int(r["Dispatch_Id"])
    e = rows.setdefault(d, {"name": re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", ""),
                            "grid": int(r["Grid_Size"]),
                            "us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
    e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
rows = list(rows.values())
starts = [i for i, r in enumerate(rows) if "nchw3_to_nhwc4" in r["name"] or "stem_patch" in r["name"]]
s = starts[-1]
e = next(i for i in range(s, len(rows)) if "kfpn_combine" in rows[i]["name"])
tot = collections.Counter()
print(f"{'kernel':60s} {'us':>7s} {'MFMA(M)':>8s} {'VALU-MFMA/MFMA':>14s} {'LDS/MFMA':>9s} {'VMEM/MFMA':>9s} {'SALU/MFMA':>9s}")
for r in rows[s:e + 1]:
    mf = r.get("SQ_INSTS_MFMA", 0)
    va = r.get("SQ_INSTS_VALU", 0) - mf
    for k in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU"):
        tot[k] += r.get(k, 0)
    d = max(mf, 1)
    print(f"{r['name'][:60]:60s} {r['us']:7.1f} {mf / 1e6:8.2f} {va / d:14.2f} {r.get('SQ_INSTS_LDS', 0) / d:9.2f} "
          f"{r.get('SQ_INSTS_VMEM_RD', 0) / d:9.2f} {r.get('SQ_INSTS_SALU', 0) / d:9.2f}")
print(json.dumps({k: v / 1e6 for k, v in tot.items()}, indent=1))
