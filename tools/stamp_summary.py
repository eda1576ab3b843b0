#!/usr/bin/env python3
"""Summarise tools/stampbench output (per-k-step s_memtime stamps of the strip kernel, round 5):
per phase of a k-step (wait for the own DMA, barrier, DMA issue + presplit, compute) the median and
mean cycles over every (block, wave, k-step), the prologue and epilogue per tile, and how many
workgroups overlap in time on a CU.

  python tools/stamp_summary.py gpurun_out/stamps_layer1.bin
"""
import sys

import numpy as np


def main(path):
    with open(path, "rb") as f:
        nb, nw, rec, nks = np.frombuffer(f.read(16), np.int32)
        d = np.frombuffer(f.read(), np.uint64).reshape(nb, nw, rec).astype(np.int64)
    t0, t1 = d[:, :, 0], d[:, :, 1]
    ks = d[:, :, 2:2 + 5 * nks].reshape(nb, nw, nks, 5)
    tend = d[:, :, 2 + 5 * 96]
    ok = (t0 > 0) & (tend > 0)
    print(f"{path}: {nb} blocks x {nw} waves, {nks} k-steps; {int(ok.sum())} complete records")
    wait = ks[..., 1] - ks[..., 0]
    bar = ks[..., 2] - ks[..., 1]
    issue = ks[..., 3] - ks[..., 2]
    comp = ks[..., 4] - ks[..., 3]
    gap = np.zeros_like(wait)
    gap[..., 1:] = ks[..., 1:, 0] - ks[..., :-1, 4]  # from one k-step's compute to the next's wait
    step = np.zeros_like(wait)
    step[..., 1:] = ks[..., 1:, 0] - ks[..., :-1, 0]
    m = ok[:, :, None] & np.ones(nks, bool)
    def st(name, x, mask=m):
        v = x[mask]
        print(f"  {name:28s} median {np.median(v):8.0f}  mean {v.mean():8.0f}  p90 {np.percentile(v, 90):8.0f} cycles")
    st("wait (own DMA landed)", wait)
    st("barrier", bar)
    st("DMA issue (+ presplit kw0)", issue)
    for kw in range(3):
        mk = m.copy()
        mk[:, :, [i for i in range(nks) if i % 3 != kw]] = False
        st(f"  issue kw {kw}", issue, mk)
    st("compute (LDS reads + MFMAs)", comp)
    for kw in range(3):
        mk = m.copy()
        mk[:, :, [i for i in range(nks) if i % 3 != kw]] = False
        st(f"  compute kw {kw}", comp, mk)
    mm = m.copy()
    mm[:, :, 0] = False
    st("k-step period", step, mm)
    pro = (t1 - t0)[ok]
    epi = (tend - ks[:, :, nks - 1, 4])[ok]
    life = (tend - t0)[ok]
    print(f"  prologue   median {np.median(pro):8.0f} cycles; epilogue median {np.median(epi):8.0f}; "
          f"tile lifetime median {np.median(life):8.0f}")
    loop = (ks[:, :, nks - 1, 4] - ks[:, :, 0, 0])[ok]
    print(f"  k-loop     median {np.median(loop):8.0f} cycles = {np.median(loop) / nks:.0f} per k-step")
    # share of the wave's lifetime per phase
    tot = life.sum()
    for name, x in (("wait", wait), ("barrier", bar), ("issue", issue), ("compute", comp), ("gap", gap)):
        print(f"  share {name:8s} {100 * x[m].sum() / tot:5.1f} %")
    print(f"  share prologue {100 * pro.sum() / tot:5.1f} %, epilogue {100 * epi.sum() / tot:5.1f} %")
    # concurrency: workgroups alive on the same CU (XCC, CU id from HW_ID bits 8..11, SH 12, SE 13..15)
    hw = d[:, 0, 2 + 5 * 96 + 1]
    cu = ((hw >> 32) << 16) | ((hw & 0xffffffff) >> 8 & 0xff)
    starts, ends = d[:, 0, 0], d[:, 0, 2 + 5 * 96]
    span = ends.max() - starts[starts > 0].min()
    print(f"  kernel span {span} cycles; sum of workgroup lifetimes / (span x distinct CUs) = "
          f"{(ends - starts)[ok[:, 0]].sum() / (span * len(np.unique(cu))):.2f} workgroups per CU on average")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
