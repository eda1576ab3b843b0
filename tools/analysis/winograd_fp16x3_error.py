"""Precision of Winograd F(2x2, 3x3) under the fp16x3 split, against the direct fp16x3 conv
(DESIGN.md §12).  CPU emulation on one level-1 head conv shape (C = 128 -> 64,
3x3, stride 1, pad 1) with He-uniform weights and ReLU-like activations, f64 reference.

fp16x3: x * s = hi + lo (s = 2^(13 - e) from max |x|, hi = fp16(x s), lo = fp16(x s - hi)); the
products hi*hi + hi*lo + lo*hi are exact in f32 and summed in f32 (the MFMA accumulator).  Direct:
the split is applied to x and to W.  Winograd: V = B^T d B (f32), U = G g G^T (f64 -> f32), each
transformed operand scaled and split per (position, channel) the same way, M_p = sum_c U_p V_p in
f32, Y = A^T M A in f32.  Prints the max |err| / max(1, |ref|) (the logit bar's metric) and the
max |err| / rms(ref) of both.

    python tools/analysis/winograd_fp16x3_error.py
"""
import numpy as np

rng = np.random.default_rng(0)
C, N, H, W = 128, 64, 32, 32


def split(v, axis_max):
    """fp16x3 terms of v with a power-of-two scale per slice along axis_max (max |v| over the rest)."""
    v = v.astype(np.float32)
    mx = np.max(np.abs(v), axis=axis_max, keepdims=True)
    e = np.floor(np.log2(np.maximum(mx, 1e-30)))
    s = np.exp2(13 - e).astype(np.float32)
    vs = v * s
    hi = vs.astype(np.float16).astype(np.float32)
    lo = (vs - hi).astype(np.float16).astype(np.float32)
    return hi, lo, s


def mm3(ah, al, bh, bl):
    """sum_k a b as three exact fp16 products accumulated in f32 (a: [..., K], b: [K, ...])."""
    f = lambda x, y: np.matmul(x.astype(np.float32), y.astype(np.float32), dtype=np.float32)  # noqa: E731
    return f(ah, bl) + f(al, bh) + f(ah, bh)


x = np.maximum(rng.standard_normal((H + 2, W + 2, C)), 0).astype(np.float32)  # padded input, ReLU-like
x[0, :] = x[-1, :] = x[:, 0] = x[:, -1] = 0
bound = np.sqrt(6.0 / (9 * C))
g = rng.uniform(-bound, bound, (N, C, 3, 3)).astype(np.float32)

# f64 reference
ref = np.zeros((H, W, N))
for kh in range(3):
    for kw in range(3):
        ref += x[kh:kh + H, kw:kw + W, :].astype(np.float64) @ g[:, :, kh, kw].T.astype(np.float64)

# direct fp16x3 (im2col over (tap, c))
cols = np.stack([x[kh:kh + H, kw:kw + W, :] for kh in range(3) for kw in range(3)], 2).reshape(H * W, 9 * C)
wmat = g.transpose(2, 3, 1, 0).reshape(9 * C, N)
xh, xl, xs = split(cols, None)
wh, wl, ws = split(wmat, 0)
direct = (mm3(xh, xl, wh, wl) / xs / ws).reshape(H, W, N)

# Winograd F(2x2, 3x3)
Bt = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float32)
Gm = np.array([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], np.float64)
At = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float32)
U = np.einsum("ij,ncjk,lk->ilnc", Gm, g.astype(np.float64), Gm).astype(np.float32)  # [4][4][N][C]
tiles = np.stack([x[2 * i:2 * i + 4, 2 * j:2 * j + 4, :] for i in range(H // 2) for j in range(W // 2)])  # [T][4][4][C]
V = np.einsum("ij,tjkc,lk->tilc", Bt, tiles, Bt, dtype=np.float32).astype(np.float32)  # [T][4][4][C]
Mp = np.zeros((tiles.shape[0], 4, 4, N), np.float32)
for a in range(4):
    for b in range(4):
        vh, vl, vs = split(V[:, a, b, :], None)
        uh, ul, us = split(U[a, b].T, 0)  # [C][N], scale per output channel
        Mp[:, a, b, :] = mm3(vh, vl, uh, ul) / vs / us
Y = np.einsum("ij,tjkn,lk->tiln", At, Mp, At, dtype=np.float32)  # [T][2][2][N]
wino = Y.reshape(H // 2, W // 2, 2, 2, N).transpose(0, 2, 1, 3, 4).reshape(H, W, N)

for name, y in (("direct fp16x3", direct), ("winograd F(2x2,3x3) fp16x3", wino)):
    err = np.abs(y - ref)
    print(f"{name:28s} max|err|/max(1,|ref|) = {np.max(err / np.maximum(1, np.abs(ref))):.3e}   "
          f"max|err|/rms(ref) = {np.max(err) / np.sqrt(np.mean(ref ** 2)):.3e}")
