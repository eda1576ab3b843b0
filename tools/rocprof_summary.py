#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (results .db or kernel_trace.csv) per kernel, per launch
shape and per forward stage; used to build the committed summaries under profiles/.

  python tools/rocprof_summary.py <run_results.db | kernel_trace.csv> [--skip-first N] [--title T]

Per forward (a forward ends at each kfpn_combine launch; the stem starts the next one):
  * conv launches = EVERY implicit-GEMM launch: conv_mfma / conv_x6(g) / conv_h3 / conv_h3s / conv_r3,
    the patch stem, the FPN kernels (fpn_gemm / fpn_row) and the split-K reduces;
  * stages, from the launches of one forward in issue order: stem (the amax memset, the stem and its
    pool merge / max-pool), layer1 .. layer4 (the body convs in order, four per layer, each split-K
    reduce with its conv), FPN + aux (every other launch up to kfpn_combine: FPN 1x1 convs, upsamples,
    KFPN combine), heads (the EPI_HEAD launches), decode (decode_* launches after the forward).
Durations are summed; launches that overlap in time (side streams, steps in flight) add up to more
than the wall time.
"""
import argparse
import collections
import csv
import re
import sqlite3

CONV_RE = re.compile(r"conv_(mfma|x6g?|h3s?|r3)_kernel|stem_patch|fpn_gemm_kernel|fpn_row_kernel|splitk_reduce")
HEAD_RE = re.compile(r"conv_r3_kernel<256, 320|conv_x6g?_kernel<[^>]*, 1, |conv_mfma_kernel<[^>]*, 1, ")
STEM_RE = re.compile(r"stem_|maxpool|fillBuffer|nchw3_to_nhwc4|amax_nhwc4")
FPN_RE = re.compile(r"fpn_|upsample|kfpn")


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
            rows = []
            for r in csv.DictReader(f):
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                rows.append(dict(name=r["Kernel_Name"], start=s, dur=e - s,
                                 grid=(r.get("Grid_Size_X"), r.get("Grid_Size_Y"), r.get("Grid_Size_Z")),
                                 wg=r.get("Workgroup_Size_X"), vgpr=r.get("VGPR_Count"),
                                 agpr=r.get("Accum_VGPR_Count"), lds=r.get("LDS_Block_Size"),
                                 cid=int(r.get("Correlation_Id") or 0)))
            # issue order: the correlation id counts dispatches in the order the host enqueued them
            rows.sort(key=lambda r: (r["cid"], r["start"]) if r["cid"] else (0, r["start"]))
            yield from rows


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = n.replace("void ", "")
    return n[:90]


def forward_stages(fwd):
    """Stage of each dispatch of one forward (a list of rows in issue order, ending at kfpn_combine)."""
    stages = []
    body = 0
    fpn_started = False
    for r in fwd:
        n = r["name"]
        if HEAD_RE.search(n):
            stages.append("heads")
        elif not fpn_started and STEM_RE.search(n):
            stages.append("stem")
        elif not fpn_started and "splitk_reduce" in n and body:
            stages.append(f"layer{(body - 1) // 4 + 1}")
        elif not fpn_started and CONV_RE.search(n) and not FPN_RE.search(n) and body < 16:
            body += 1
            stages.append(f"layer{(body - 1) // 4 + 1}")
        else:
            fpn_started = True
            stages.append("fpn+aux")
    return stages


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--skip-first", type=int, default=0, help="drop the first N dispatches (warm-up)")
    ap.add_argument("--title", default=None, help="first line of the summary (the command it profiles)")
    a = ap.parse_args()
    rows = list(rows_from(a.path))[a.skip_first:]
    if a.title:
        print(f"# {a.title}")
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
    ends = [i for i, r in enumerate(rows) if "kfpn_combine" in r["name"]]
    if ends:
        nf = len(ends)
        conv = sum(r["dur"] for r in rows if CONV_RE.search(r["name"]))
        aux = sum(r["dur"] for r in rows if re.search(r"maxpool|upsample|nchw3|kfpn|fillBuffer", r["name"]))
        dec = sum(r["dur"] for r in rows if "decode_" in r["name"])
        print(f"# forwards: {nf}; per forward: conv launches (every implicit-GEMM kernel, split-K reduces "
              f"included) {conv / nf / 1e3:.1f} us, memset/maxpool/upsample/layout/kfpn {aux / nf / 1e3:.1f} us, "
              f"decode {dec / nf / 1e3:.1f} us (durations summed; concurrent launches overlap in wall time)")
        # per-stage sums over every complete forward (from the first stem launch after a kfpn_combine)
        starts = [0] + [e + 1 for e in ends[:-1]]
        stage_tot = collections.OrderedDict((s, 0) for s in
                                            ("stem", "layer1", "layer2", "layer3", "layer4", "fpn+aux", "heads", "decode"))
        nfull = 0
        for lo, hi in zip(starts, ends):
            fwd = rows[lo:hi + 1]
            first = next((i for i, r in enumerate(fwd) if STEM_RE.search(r["name"])), None)
            if first is None:
                continue
            fwd = fwd[first:]
            nfull += 1
            for r, s in zip(fwd, forward_stages(fwd)):
                stage_tot[s] += r["dur"]
            # the decode launches that follow this forward (before the next forward's stem)
            j = hi + 1
            while j < len(rows) and "decode_" in rows[j]["name"]:
                stage_tot["decode"] += rows[j]["dur"]
                j += 1
        if nfull:
            s_all = sum(stage_tot.values())
            print(f"# per-stage kernel time per forward (mean of {nfull} forwards; sum {s_all / nfull / 1e3:.1f} us):")
            for s, v in stage_tot.items():
                print(f"#   {s:8s} {v / nfull / 1e3:9.1f} us  {100 * v / max(s_all, 1):5.1f} %")
        if len(ends) >= 2:
            lo, hi = ends[-2] + 1, ends[-1] + 1
            fwd = rows[lo:hi]
            first = next((i for i, r in enumerate(fwd) if STEM_RE.search(r["name"])), 0)
            fwd = fwd[first:]
            t0 = fwd[0]["start"]
            print("\n# one forward in issue order (start offset us, duration us, stage)")
            for r, s in zip(fwd, forward_stages(fwd)):
                print(f"{(r['start'] - t0) / 1e3:9.1f} {r['dur'] / 1e3:9.1f}  {s:8s} {short(r['name'])[:70]:70s} {r['grid']}")
    print("\n# per launch shape (grid = total work-items)")
    print(f"{'kernel':90s} {'grid':>22s} {'calls':>6s} {'avg_us':>10s}")
    for (k, g), d in sorted(by_shape.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:90s} {str(g):>22s} {len(d):6d} {sum(d) / len(d) / 1e3:10.2f}")


if __name__ == "__main__":
    main()
