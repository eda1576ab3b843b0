#!/usr/bin/env python3
"""HBM bytes of one sfa_bev_voxelize call (the blocked path's bin / strip kernels, or round 2's
binned count / scan / bin / strip)
from tools/pmc_bev.sh output -> JSON for profiles/. FETCH_SIZE doubled and WRITE_SIZE as is
(gfx950 corrections, MI355X_MICROARCH.md §HBM); the last call of the run is summarised.

  python tools/pmc_bev_summary.py gpurun_out/pmc_bev profiles/r02c_pmc_bev.json"""
import csv, collections, hashlib, json, os, re, sys

base, out = sys.argv[1], sys.argv[2]
KERNELS = ("bev_bin_count_kernel", "bev_bin_scan_kernel", "bev_bin_kernel", "bev_strip_kernel",
           "bev_blk_bin_kernel", "bev_blk_strip_kernel")
FIRST = ("bev_bin_count_kernel", "bev_blk_bin_kernel")  # the first kernel of a call


def load(p, counter):
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(os.path.join(base, p, "run_counter_collection.csv"))):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        if not any(k + "<" in name or name.endswith(k) for k in KERNELS) or r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        e = rows.setdefault(d, {"name": name, "dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), "v": 0.0})
        e["v"] += float(r["Counter_Value"])
    return list(rows.values())


fetch, write = load("p1", "FETCH_SIZE"), load("p2", "WRITE_SIZE")
# the last call: the dispatches from the last first-kernel on (blocked: bin, strip; round 2's
# binned: count, scan, bin, strip)
def last_call(rows):
    starts = [i for i, r in enumerate(rows) if any(k + "<" in r["name"] or r["name"].endswith(k) for k in FIRST)]
    return rows[starts[-1]:]


f4, w4 = last_call(fetch), last_call(write)
assert [r["name"] for r in f4] == [r["name"] for r in w4], (f4, w4)
per = [{"kernel": f["name"], "us": f["dur_ns"] / 1e3, "fetch_MB": 2 * f["v"] * 1024 / 1e6,
        "write_MB": w["v"] * 1024 / 1e6} for f, w in zip(f4, w4)]
total = sum(r["fetch_MB"] + r["write_MB"] for r in per) * 1e6
res = {"bev_hbm_bytes_per_call": int(total), "per_kernel": per,
       "method": "rocprofv3 --kernel-trace --pmc (FETCH_SIZE, WRITE_SIZE passes), bench.py --workload e2e --no-graph; "
                 "HBM = 2*FETCH_SIZE + WRITE_SIZE (KiB), last sfa_bev_voxelize call (16 sweeps)",
       "kernels": [r["kernel"] for r in per]}
_lib = os.environ.get("SFA_HIP_LIB") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
    "lidar-image_object-detection_-fpn_resnet-yolov8_amd", "sfa", "sfa_hip", "libsfa_hip.so")
res["lib_sha256"] = hashlib.sha256(open(_lib, "rb").read()).hexdigest()  # bench.py matches it
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
