#!/usr/bin/env python3
"""Summarise tools/headstampbench output (s_memtime stamps of the fused heads kernel, round 5): per
wave the prologue (start -> after the first barrier), the K loop and the epilogue; the K-tile memory waits (vmcnt) and
barriers by wave half; and per CU the idle gap between one tile's last wave ending and the next tile's first wave
starting (block turnover), as shares of the CU's busy time.

  python tools/head_stamp_summary.py gpurun_out/hstamps_L1.bin
"""
import sys

import numpy as np

NKT_MAX = 40


def main(path):
    with open(path, "rb") as f:
        nb, nw, rec, nkt = np.frombuffer(f.read(16), np.int32)
        d = np.frombuffer(f.read(), np.uint64).reshape(nb, nw, rec).astype(np.int64)
    t0, t1, t2, t3 = (d[:, :, i] for i in range(4))
    ok = (t0 > 0) & (t3 > 0)
    print(f"{path}: {nb} tiles x {nw} waves, {nkt} K-tiles; {int(ok.sum())} complete records")
    pro, loop, epi, life = (t1 - t0)[ok], (t2 - t1)[ok], (t3 - t2)[ok], (t3 - t0)[ok]
    def st(name, v):
        print(f"  {name:26s} median {np.median(v):9.0f}  mean {v.mean():9.0f}  p90 {np.percentile(v, 90):9.0f} cycles")
    st("prologue", pro)
    st("K loop", loop)
    st("  per K-tile", loop / nkt)
    st("epilogue", epi)
    st("tile lifetime (wave)", life)
    k = min(nkt, NKT_MAX)
    vw = (d[:, :, 6:6 + 3 * k:3] - d[:, :, 5:5 + 3 * k:3])
    bw = (d[:, :, 7:7 + 3 * k:3] - d[:, :, 6:6 + 3 * k:3])
    for half, sel in (("leading half", slice(0, nw // 2)), ("delayed half", slice(nw // 2, nw))):
        okh = ok[:, sel]
        st(f"memory wait, {half}", vw[:, sel][okh].reshape(-1))
        st(f"barrier, {half}", bw[:, sel][okh].reshape(-1))
    vws, bws = vw[ok].sum() * nkt / k, bw[ok].sum() * nkt / k
    print(f"  shares of the waves' lifetimes: prologue {100 * pro.sum() / life.sum():.1f} %, K loop "
          f"{100 * loop.sum() / life.sum():.1f} % (memory waits ~{100 * vws / life.sum():.1f} %, barriers "
          f"~{100 * bws / life.sum():.1f} %), epilogue {100 * epi.sum() / life.sum():.1f} %")
    # per CU: tiles in start order, the gap from a tile's end (last wave) to the next tile's start (first wave)
    hw = d[:, 0, 4]
    cu = ((hw >> 32) << 16) | ((hw & 0xffffffff) >> 8 & 0xff)
    okb = ok.all(axis=1)
    starts, ends = t0.min(axis=1), t3.max(axis=1)
    gaps, busy, first = [], 0, []
    for c in np.unique(cu[okb]):
        idx = np.where((cu == c) & okb)[0]
        idx = idx[np.argsort(starts[idx])]
        s, e = starts[idx], ends[idx]
        busy += int((e - s).sum())
        if len(idx) > 1:
            gaps.extend((s[1:] - e[:-1]).tolist())
        first.append(len(idx))
    gaps = np.array(gaps)
    print(f"  CUs {len(first)}, tiles per CU {min(first)}..{max(first)}; turnover gap median {np.median(gaps):.0f} "
          f"cycles (p90 {np.percentile(gaps, 90):.0f}, negative = overlap), sum of gaps / sum of tile lifetimes "
          f"{100 * np.clip(gaps, 0, None).sum() / busy:.1f} %")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
