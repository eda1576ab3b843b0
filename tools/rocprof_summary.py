#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (results .db or kernel_trace.csv) per kernel
and per launch shape; used to build the committed summaries under profiles/.

  python tools/rocprof_summary.py <run_results.db | kernel_trace.csv> [--skip-first N]
"""
import argparse
import collections
import csv
import re
import sqlite3


def rows_from(path):
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        cur = con.cursor()
        for name, s, e, gx, gy, gz, wx, vg, ag, lds in cur.execute(
                "select name, start, end, grid_x, grid_y, grid_z, workgroup_x, vgpr_count, "
                "accum_vgpr_count, lds_size from kernels order by start"):
            yield dict(name=name, start=s, dur=e - s, grid=(gx, gy, gz), wg=wx, vgpr=vg, agpr=ag, lds=lds)
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                yield dict(name=r["Kernel_Name"], start=s, dur=e - s,
                           grid=(r.get("Grid_Size_X"), r.get("Grid_Size_Y"), r.get("Grid_Size_Z")),
                           wg=r.get("Workgroup_Size_X"), vgpr=r.get("VGPR_Count"),
                           agpr=r.get("Accum_VGPR_Count"), lds=r.get("LDS_Block_Size"))


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = n.replace("void ", "")
    return n[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--skip-first", type=int, default=0, help="drop the first N dispatches (warm-up)")
    a = ap.parse_args()
    rows = list(rows_from(a.path))[a.skip_first:]
    by_kernel = collections.defaultdict(list)
    by_shape = collections.defaultdict(list)
    for r in rows:
        by_kernel[short(r["name"])].append(r["dur"])
        by_shape[(short(r["name"]), r["grid"])].append(r["dur"])
    total = sum(r["dur"] for r in rows)
    print(f"# {len(rows)} dispatches, {total / 1e6:.3f} ms total kernel time")
    print(f"{'kernel':90s} {'calls':>6s} {'avg_us':>10s} {'total_ms':>10s} {'pct':>6s}")
    for k, d in sorted(by_kernel.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:90s} {len(d):6d} {sum(d) / len(d) / 1e3:10.2f} {sum(d) / 1e6:10.3f} "
              f"{100 * sum(d) / total:6.2f}")
    # per forward: a forward starts at each kfpn-input conversion / stem launch and ends
    # at kfpn_combine; conv = every implicit-GEMM launch
    fwd = [r for r in rows if "kfpn_combine" in r["name"]]
    if fwd:
        nf = len(fwd)
        conv = sum(r["dur"] for r in rows if re.search(r"conv_(mfma|x6g?|h3)_kernel", r["name"]))
        aux = sum(r["dur"] for r in rows if re.search(r"maxpool|upsample|nchw3|kfpn", r["name"]))
        print(f"# forwards: {nf}; per forward: conv launches {conv / nf / 1e3:.1f} us, "
              f"maxpool/upsample/layout/kfpn {aux / nf / 1e3:.1f} us "
              f"(durations summed; concurrent launches overlap in wall time)")
        # the dispatches of one forward in issue order (the one before the last kfpn_combine)
        ends = [i for i, r in enumerate(rows) if "kfpn_combine" in r["name"]]
        if len(ends) >= 2:
            lo, hi = ends[-2] + 1, ends[-1] + 1
            t0 = rows[lo]["start"]
            print("\n# one forward in issue order (start offset us, duration us)")
            for r in rows[lo:hi]:
                print(f"{(r['start'] - t0) / 1e3:9.1f} {r['dur'] / 1e3:9.1f}  {short(r['name'])[:70]:70s} {r['grid']}")
    print("\n# per launch shape (grid = total work-items)")
    print(f"{'kernel':90s} {'grid':>22s} {'calls':>6s} {'avg_us':>10s}")
    for (k, g), d in sorted(by_shape.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:90s} {str(g):>22s} {len(d):6d} {sum(d) / len(d) / 1e3:10.2f}")


if __name__ == "__main__":
    main()
