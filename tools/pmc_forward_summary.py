#!/usr/bin/env python3
"""Per-forward HBM traffic from tools/pmc_forward.sh output -> JSON for profiles/.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports half the
bytes of a wide (16 B/lane) coalesced read -> doubled; WRITE_SIZE (KiB) taken as is.
The last forward of the run (the one after warm-up) is summarised."""
import csv, collections, hashlib, json, os, re, sys

base = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else None


def load(p):
    f = os.path.join(base, p, "run_counter_collection.csv")
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        d = int(r["Dispatch_Id"])
        e = rows.setdefault(d, {"name": re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", ""),
                                "grid": int(r["Grid_Size"]),
                                "dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(rows.values())


passes = [load(p) for p in sorted(d for d in os.listdir(base) if d.startswith("p") and
                                  os.path.isdir(os.path.join(base, d)))]
# dispatches are matched across passes by (kernel, grid, occurrence): with the level-0
# heads on a side stream the dispatch order differs from pass to pass
def keyed(p):
    seen = collections.Counter()
    out = {}
    for r in p:
        k = (r["name"], r["grid"])
        out[k + (seen[k],)] = r
        seen[k] += 1
    return out


keyed_passes = [keyed(p) for p in passes[1:]]
merged = []
seen = collections.Counter()
for r0 in passes[0]:
    k = (r0["name"], r0["grid"])
    key = k + (seen[k],)
    seen[k] += 1
    if not all(key in kp for kp in keyed_passes):
        continue
    row = dict(r0)
    for kp in keyed_passes:
        row.update({k2: v for k2, v in kp[key].items() if k2 not in ("name", "grid", "dur_ns")})
    merged.append(row)
# last forward: from its first kernel (the layout pass until round 3, the stem since the stem reads
# the input layout itself) to the following kfpn_combine
starts = [i for i, r in enumerate(merged) if "nchw3_to_nhwc4" in r["name"]]
if not starts:
    starts = [i for i, r in enumerate(merged) if "stem_patch_pool" in r["name"]]
s = starts[-1]
e = next(i for i in range(s, len(merged)) if "kfpn_combine" in merged[i]["name"])
fwd = merged[s:e + 1]
conv = [r for r in fwd if re.search(r"conv_(mfma|x6g?|h3s?|r3)_kernel|splitk_reduce|stem_patch", r["name"])]


def hbm(r):
    return 2 * r.get("FETCH_SIZE", 0) * 1024 + r.get("WRITE_SIZE", 0) * 1024


res = {
    "conv_launches": len(conv),
    "conv_hbm_bytes_per_forward": sum(hbm(r) for r in conv),
    "conv_fetch_bytes_corrected": sum(2 * r.get("FETCH_SIZE", 0) * 1024 for r in conv),
    "conv_write_bytes": sum(r.get("WRITE_SIZE", 0) * 1024 for r in conv),
    "forward_hbm_bytes": sum(hbm(r) for r in fwd),
    "conv_l2_hit_rate": sum(r.get("TCC_HIT_sum", 0) for r in conv) /
    max(1.0, sum(r.get("TCC_HIT_sum", 0) + r.get("TCC_MISS_sum", 0) for r in conv)),
    "conv_mfma_busy_frac": sum(r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for r in conv) /
    max(1.0, sum(r.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024 for r in conv)),
    "effective_clock_ghz": sum(r.get("GRBM_GUI_ACTIVE", 0) / 8 for r in conv) /
    max(1.0, sum(r["dur_ns"] for r in conv)),
    "per_launch": [{"kernel": r["name"], "grid": r["grid"], "us": r["dur_ns"] / 1e3,
                    "hbm_MB": hbm(r) / 1e6,
                    "mfma_busy": r.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) /
                    max(1.0, r.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024)} for r in fwd],
    "method": "rocprofv3 --kernel-trace --pmc, one counter group per pass, bench.py --no-graph; "
              "HBM = 2*FETCH_SIZE + WRITE_SIZE (KiB, gfx950 FETCH_SIZE halving corrected)",
}
# the library build the passes ran (bench.py reports this file's traffic only for the same build)
_lib = os.environ.get("SFA_HIP_LIB") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
    "lidar-image_object-detection_-fpn_resnet-yolov8_amd", "sfa", "sfa_hip", "libsfa_hip.so")
res["lib_sha256"] = hashlib.sha256(open(_lib, "rb").read()).hexdigest()
txt = json.dumps(res, indent=1)
if out:
    open(out, "w").write(txt)
print(txt[:3000])
