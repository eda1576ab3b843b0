#!/usr/bin/env python3
"""Per-launch roofline table of one 608x608, bs=16 forward, from committed evidence only.

Inputs (no GPU needed):
  * a serial rocprof summary (tools/rocprof_summary.py output: "one forward in issue order" maps
    each launch to its kernel and grid; "per launch shape" gives the mean duration per kernel and grid
    over every timed forward),
  * the PMC traffic pass of the same library build (tools/pmc_forward_summary.py: HBM bytes and MFMA
    busy per launch, in issue order),
  * a bench.py line (its heads probe splits the three heads launches, which share one template and,
    for levels 1 and 2, one grid).

Algorithmic FLOP per launch are the reference's (fpn_resnet_18 at 608^2): 2 M N K of
the conv the launch computes, K including a fused 1x1 downsample; an FPN pair (the commuted 1x1:
low-resolution W_a x + the skip conv with the upsampled residual) is charged the reference's
1x1 conv on the upsampled concat, split over its two launches by their durations. The sum is
bench.py's CONV_FLOP_PER_FRAME x 16.  Peaks: fp16x3 833.3 TFLOP/s (2.5 PF dense fp16 / 3 products),
HBM 8 TB/s (MI355X_MICROARCH.md).

usage: tools/stage_rooflines.py SUMMARY.txt PMC.json BENCH.json [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import re
import sys

B, H, W = 16, 608, 608
PEAK_TF = 2500.0 / 3
PEAK_TBS = 8.0


def conv_flop(m, n, k):
    return 2.0 * m * n * k


def forward_plan():
    """(stage, label, flop or None, pair id) per launch, in the forward's issue order (model.hip)."""
    s4, s8, s16, s32 = (B * (H // d) * (W // d) for d in (4, 8, 16, 32))
    s2 = B * (H // 2) * (W // 2)
    plan = [("stem", "conv1 7x7/2 3->64 + bn + relu + maxpool", conv_flop(s2, 64, 147), None),
            ("stem", "maxpool halo merge", None, None)]
    plan += [("layer1", "layer1.%d.conv%d 3x3 64->64" % (i // 2, i % 2 + 1), conv_flop(s4, 64, 576), None)
             for i in range(4)]
    for li, (m, cin, cout) in enumerate(((s8, 64, 128), (s16, 128, 256), (s32, 256, 512)), start=2):
        st = "layer%d" % li
        plan.append((st, "%s.0.conv1 3x3/2 %d->%d" % (st, cin, cout), conv_flop(m, cout, 9 * cin), None))
        if li == 4:
            plan.append((st, "split-K reduce", None, None))
        plan.append((st, "%s.0.conv2 3x3 + downsample 1x1/2" % st, conv_flop(m, cout, 9 * cout + cin), None))
        if li == 4:
            plan.append((st, "split-K reduce", None, None))
        plan += [(st, "%s.1.conv%d 3x3 %d->%d" % (st, j + 1, cout, cout), conv_flop(m, cout, 9 * cout), None)
                 for j in range(2)]
    up1 = conv_flop(s16, 256, 512 + 256)   # conv_up_level1 on cat(up(layer4), layer3)
    up2 = conv_flop(s8, 128, 256 + 128)    # conv_up_level2 on cat(up(c1), layer2)
    up3 = conv_flop(s4, 64, 128 + 64)      # conv_up_level3 on cat(up(c2), layer1)
    heads = lambda m, c: conv_flop(m, 320, 9 * c) + conv_flop(m, 11, 64 * 1)  # 3x3 C->5x64 + 1x1s
    plan += [("fpn+aux", "conv_up_level1: W_a layer4 (low res)", up1, 1),
             ("fpn+aux", "conv_up_level1: skip conv + upsampled residual", up1, 1),
             ("fpn+aux", "upsample c1 -> up_level2", None, None),
             ("heads", "heads level 0 (up_level2, 256 ch, 76^2)", None, "h0"),
             ("fpn+aux", "conv_up_level2: W_a c1 (low res)", up2, 2),
             ("fpn+aux", "conv_up_level2: skip conv + upsampled residual", up2, 2),
             ("fpn+aux", "upsample c2 -> up_level3", None, None),
             ("fpn+aux", "conv_up_level3: W_a c2 (low res)", up3, 3),
             ("fpn+aux", "conv_up_level3: skip conv + upsampled residual", up3, 3),
             ("heads", "heads level 1 (up_level3, 128 ch, 152^2)", None, "h1"),
             ("heads", "heads level 2 (up_level4, 64 ch, 152^2)", None, "h2"),
             ("fpn+aux", "apply_kfpn", None, None)]
    return plan


def parse_summary(path):
    issue, shapes = [], {}
    sec = None
    for line in open(path):
        if line.startswith("# one forward in issue order"):
            sec = "issue"
            continue
        if line.startswith("# per launch shape"):
            sec = "shape"
            continue
        if sec == "issue":
            m = re.match(r"\s*([\d.]+)\s+([\d.]+)\s+(\S+)\s+(.*?)\s+(\('\d+'.*\))\s*$", line)
            if m:
                issue.append((m.group(4).strip(), m.group(5)))
            elif issue and not line.strip():
                sec = None
        elif sec == "shape":
            m = re.match(r"(sfa::.*?)\s+(\('\d+'.*?\))\s+(\d+)\s+([\d.]+)\s*$", line)
            if m:
                shapes[(m.group(1).strip(), m.group(2))] = float(m.group(4))
    return issue, shapes


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("summary")
    ap.add_argument("pmc")
    ap.add_argument("bench")
    ap.add_argument("--out")
    args = ap.parse_args(argv)
    issue, shapes = parse_summary(args.summary)
    pmc = json.load(open(args.pmc))
    per = pmc["per_launch"]
    bench = json.loads(open(args.bench).readline())
    head_us = bench["roofline"]["launch_us"]
    head_flop = bench["roofline"]["algorithmic_flop_per_launch"]
    plan = forward_plan()
    if not (len(issue) == len(per) == len(plan)):
        sys.exit("launch counts differ: summary %d, PMC %d, plan %d" % (len(issue), len(per), len(plan)))
    rows = []
    for i, ((kname, grid), p, (stage, label, flop, pair)) in enumerate(zip(issue, per, plan)):
        if not p["kernel"].startswith(kname[:40]):
            sys.exit("launch %d: summary kernel %s vs PMC %s" % (i, kname, p["kernel"]))
        cands = [v for (k, g), v in shapes.items() if g == grid and k.startswith(kname)]
        us = cands[0] if len(cands) == 1 else None
        if isinstance(pair, str):  # heads: the bench's per-level probe
            lvl = int(pair[1])
            us, flop = head_us[lvl], head_flop[lvl]
        rows.append(dict(i=i, stage=stage, label=label, kernel=p["kernel"], grid=grid, us=us, flop=flop,
                         pair=pair, hbm=p["hbm_MB"] * 1e6, busy=p["mfma_busy"]))
    for pid in (1, 2, 3):  # FPN pairs: the reference conv's FLOP split by duration
        pr = [r for r in rows if r["pair"] == pid]
        tot = sum(r["us"] for r in pr)
        for r in pr:
            r["flop"] = r["flop"] * r["us"] / tot
    out = []
    pr = out.append
    pr("# per-launch rooflines of one forward (bs=16, 3x608x608, fp16x3), from %s + %s + %s"
       % (args.summary, args.pmc, args.bench))
    pr("# us: serial rocprof mean per kernel and grid (heads: bench probe per level); GF: reference"
       " algorithmic FLOP; TF/s and frac vs the fp16x3 peak %.1f; HBM: PMC bytes of this library build"
       " (sha256 %s); TB/s and frac vs %.0f TB/s" % (PEAK_TF, pmc.get("lib_sha256", "?")[:16], PEAK_TBS))
    pr("%-3s %-8s %-48s %8s %8s %7s %6s %8s %6s %5s %5s" % ("#", "stage", "launch", "us", "GFLOP", "TF/s",
                                                          "frac", "HBM MB", "TB/s", "frac", "mfma"))
    stage_sum = {}
    for r in rows:
        tf = r["flop"] / (r["us"] * 1e-6) / 1e12 if r["flop"] else None
        tbs = r["hbm"] / (r["us"] * 1e-6) / 1e12
        bound = "mfma" if r["flop"] else "hbm"
        pr("%-3d %-8s %-48s %8.1f %8s %7s %6s %8.1f %6.2f %5.2f %5.2f  %s"
           % (r["i"], r["stage"], r["label"][:48], r["us"], "%.2f" % (r["flop"] / 1e9) if r["flop"] else "-",
              "%.1f" % tf if tf else "-", "%.3f" % (tf / PEAK_TF) if tf else "-", r["hbm"] / 1e6, tbs,
              tbs / PEAK_TBS, r["busy"], bound))
        s = stage_sum.setdefault(r["stage"], [0.0, 0.0, 0.0])
        s[0] += r["us"]
        s[1] += r["flop"] or 0.0
        s[2] += r["hbm"]
    pr("")
    pr("# per stage (launch durations summed; concurrent launches overlap in the timed loop)")
    pr("%-8s %9s %9s %7s %6s %9s" % ("stage", "us", "GFLOP", "TF/s", "frac", "HBM MB"))
    tot = [0.0, 0.0, 0.0]
    for st, (us, fl, hb) in stage_sum.items():
        pr("%-8s %9.1f %9.2f %7.1f %6.3f %9.1f" % (st, us, fl / 1e9, fl / (us * 1e-6) / 1e12,
                                                  fl / (us * 1e-6) / 1e12 / PEAK_TF, hb / 1e6))
        tot = [a + b for a, b in zip(tot, (us, fl, hb))]
    pr("%-8s %9.1f %9.2f %7.1f %6.3f %9.1f" % ("forward", tot[0], tot[1] / 1e9, tot[1] / (tot[0] * 1e-6) / 1e12,
                                              tot[1] / (tot[0] * 1e-6) / 1e12 / PEAK_TF, tot[2] / 1e6))
    text = "\n".join(out) + "\n"
    if args.out:
        open(args.out, "w").write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
