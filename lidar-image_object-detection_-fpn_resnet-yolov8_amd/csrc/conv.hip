// Implicit-GEMM convolution on fp32 MFMA for gfx950 (CDNA4).
//
// Every convolution of the KFPN forward (models/fpn_resnet.py:37-145, 53 convs,
// 62.57 GFLOP/frame) runs here as C[M][N] = A[M][K] * W[N][K]^T with
//   M = B*OH*OW output pixels (NHWC rows), N = Cout, K = taps*Cin (+ a 2nd segment).
// The A tile is gathered straight from the NHWC activation (no im2col buffer);
// BatchNorm is folded into W / bias on the host; bias, residual add and ReLU
// are fused into the epilogue; a downsample 1x1 conv is fused as a second
// K-segment; the detection heads' 1x1 convs run in the EPI_HEAD epilogue.
//
// MFMA: v_mfma_f32_32x32x2_f32 (exact f32 FMA chain, 64 FLOP/clk/SIMD — the
// fp32 matrix peak, 157.3 TF).  Lane l = (r = l&31, h = l>>5) feeds A[row r]
// and B[col r] at k-slot h; at k-step s the slot-h lanes carry actual k = 8h+s,
// so each lane reads 8 contiguous k of its row (2 x ds_read_b128) for a whole
// BK = 16 tile.  LDS rows are padded to 20 floats: any 16 rows hit 16 distinct
// 16-B bank groups, so the b128 fragment reads are conflict-free.
#include "conv.h"

namespace sfa {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBK = 16;
constexpr int kLDK = kBK + 4;

template <int BM, int BN, int WM, int WN, int EPI>
__global__ void __launch_bounds__(256, 2) conv_mfma_kernel(const ConvArgs a) {
  constexpr int WAVES_N = BN / WN;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per block");
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int A_LD = BM / 64, B_LD = BN / 64;
  constexpr int STAGE = (BM + BN) * kLDK;
  constexpr int HEAD_LDS = EPI == EPI_HEAD ? BM * 65 : 0;
  constexpr int LDS_FLOATS = (2 * STAGE > HEAD_LDS) ? 2 * STAGE : HEAD_LDS;
  __shared__ __attribute__((aligned(16))) float smem[LDS_FLOATS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int n_tiles = a.N / BN;
  const int lbid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lbid / n_tiles, nt = lbid - mt * n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int M = a.M;

  // ---- loader geometry: thread -> (row rr + 64 i, k-quad kq)
  const int kq = tid & 3, rr = tid >> 2;
  int a_b[A_LD], a_oh[A_LD], a_ow[A_LD];
  bool a_ok[A_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int m = m0 + rr + 64 * i;
    a_ok[i] = m < M;
    const int mm = a_ok[i] ? m : 0;
    const int ow = mm % a.OW;
    const int t = mm / a.OW;
    a_ow[i] = ow;
    a_oh[i] = t % a.OH;
    a_b[i] = t / a.OH;
  }

  f32x4 ra[A_LD], rb[B_LD];
  auto load_tile = [&](int kt) {
    const int k0 = kt * kBK;
    const bool s1 = a.nseg > 1 && k0 >= a.kseg1;
    const float* x = s1 ? a.seg[1].x : a.seg[0].x;
    const int H = s1 ? a.seg[1].H : a.seg[0].H;
    const int W = s1 ? a.seg[1].W : a.seg[0].W;
    const int C = s1 ? a.seg[1].C : a.seg[0].C;
    const int logC = s1 ? a.seg[1].logC : a.seg[0].logC;
    const int KW = s1 ? a.seg[1].KW : a.seg[0].KW;
    const int stride = s1 ? a.seg[1].stride : a.seg[0].stride;
    const int pad = s1 ? a.seg[1].pad : a.seg[0].pad;
    const int taps = s1 ? a.seg[1].taps : a.seg[0].taps;
    const int kl = k0 - (s1 ? a.kseg1 : 0) + 4 * kq;
    const int tap = kl >> logC;
    const int c = kl & (C - 1);
    const int kh = tap / KW;
    const int kw = tap - kh * KW;
    const bool tap_ok = tap < taps;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int ih = a_oh[i] * stride - pad + kh;
      const int iw = a_ow[i] * stride - pad + kw;
      const bool ok = a_ok[i] && tap_ok && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      if (ok) {
        const size_t off = ((((size_t)a_b[i] * H + ih) * W + iw) << logC) + c;
        ra[i] = *reinterpret_cast<const f32x4*>(x + off);
      } else {
        ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      const int n = n0 + rr + 64 * j;
      rb[j] = *reinterpret_cast<const f32x4*>(a.w + (size_t)n * a.Kpad + k0 + 4 * kq);
    }
  };
  auto store_tile = [&](int stage) {
    float* As = smem + stage * STAGE;
    float* Bs = As + BM * kLDK;
#pragma unroll
    for (int i = 0; i < A_LD; ++i)
      *reinterpret_cast<f32x4*>(As + (rr + 64 * i) * kLDK + 4 * kq) = ra[i];
#pragma unroll
    for (int j = 0; j < B_LD; ++j)
      *reinterpret_cast<f32x4*>(Bs + (rr + 64 * j) * kLDK + 4 * kq) = rb[j];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[mi][ni][v] = 0.f;

  const int r = lane & 31, h = lane >> 5;
  auto compute = [&](int stage) {
    const float* As = smem + stage * STAGE;
    const float* Bs = As + BM * kLDK;
    f32x4 af[TM][2], bf[TN][2];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const float* p = As + (wm * WM + mi * 32 + r) * kLDK + 8 * h;
      af[mi][0] = *reinterpret_cast<const f32x4*>(p);
      af[mi][1] = *reinterpret_cast<const f32x4*>(p + 4);
    }
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const float* p = Bs + (wn * WN + ni * 32 + r) * kLDK + 8 * h;
      bf[ni][0] = *reinterpret_cast<const f32x4*>(p);
      bf[ni][1] = *reinterpret_cast<const f32x4*>(p + 4);
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        const float av = af[mi][s >> 2][s & 3];
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const float bv = bf[ni][s >> 2][s & 3];
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[mi][ni], 0, 0, 0);
        }
      }
    }
  };

  const int nk = a.Kpad / kBK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // Unconditional prefetch (the last iteration re-stages the final tile into the
    // idle buffer): keeps ra/rb in registers — a conditional definition made hipcc
    // spill them to scratch.
    load_tile(kt + 1 < nk ? kt + 1 : kt);
    compute(cur);
    store_tile(cur ^ 1);
    __syncthreads();
  }

  if constexpr (EPI == EPI_STD) {
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int n = n0 + wn * WN + ni * 32 + r;
      const float bn = a.bias[n];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int m = m0 + wm * WM + mi * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
          if (m < M) {
            float val = acc[mi][ni][v] + bn;
            if (a.res) val += a.res[(size_t)m * a.N + n];
            if (a.relu) val = fmaxf(val, 0.f);
            a.y[(size_t)m * a.N + n] = val;
          }
        }
      }
    }
  } else {
    // Detection head: ReLU(conv3x3 + b) staged in LDS, then the head's 1x1 conv.
    static_assert(BN == 64, "one head (head_conv = 64 channels) per block column");
    float* T = smem;  // [BM][65]; the K-loop's final barrier retired every LDS read
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int col = wn * WN + ni * 32 + r;
      const float bn = a.bias[n0 + col];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int row = wm * WM + mi * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
          T[row * 65 + col] = fmaxf(acc[mi][ni][v] + bn, 0.f);
        }
    }
    __syncthreads();
    int ch = 0, hoff = 0;
#pragma unroll
    for (int j = 0; j < SFA_MAX_HEADS; ++j)
      if (j == nt) {
        ch = a.hch[j];
        hoff = a.hoff[j];
      }
    for (int idx = tid; idx < BM * ch; idx += 256) {
      const int row = idx % BM, c = idx / BM;
      const int m = m0 + row;
      if (m >= M) continue;
      const float* wr = a.hw1 + (nt * 4 + c) * 64;
      float s = a.hb1[nt * 4 + c];
      const float* tr = T + row * 65;
#pragma unroll 16
      for (int k = 0; k < 64; ++k) s = fmaf(tr[k], wr[k], s);
      a.hout[(size_t)(hoff + c) * M + m] = s;
    }
  }
}

template <int BM, int BN, int WM, int WN, int EPI>
static int launch_cfg(const ConvArgs& a, hipStream_t st) {
  const int mt = ceil_div(a.M, BM);
  const int nt = a.N / BN;
  const long long nblocks = (long long)mt * nt;
  if (nblocks <= 0 || nblocks > 0x7fffffffll) {
    set_error("conv: bad grid (M=%d N=%d)", a.M, a.N);
    return SFA_E_INVALID;
  }
  hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, WN, EPI>), dim3((unsigned)nblocks), dim3(256), 0,
                     st, a);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

int launch_conv(const ConvArgs& a, int epilogue, hipStream_t st) {
  // Host-side shape checks: the kernels assume these and never bounds-check them.
  if (a.N <= 0 || a.N % 64 != 0 || a.M <= 0 || a.Kpad <= 0 || a.Kpad % kBK != 0) {
    set_error("conv: unsupported shape M=%d N=%d Kpad=%d", a.M, a.N, a.Kpad);
    return SFA_E_UNSUPPORTED;
  }
  for (int s = 0; s < a.nseg; ++s) {
    const ConvSeg& g = a.seg[s];
    if (!g.x || g.C < 4 || (g.C & (g.C - 1)) || (1 << g.logC) != g.C || g.KW <= 0 || g.KH <= 0) {
      set_error("conv: bad segment %d (C=%d)", s, g.C);
      return SFA_E_UNSUPPORTED;
    }
    if (g.C < kBK && s != a.nseg - 1) {
      set_error("conv: narrow-channel segment must be last");
      return SFA_E_UNSUPPORTED;
    }
  }
  if (a.nseg == 2 && (a.kseg1 % kBK != 0 || a.kseg1 <= 0 || a.kseg1 >= a.Kpad)) {
    set_error("conv: bad kseg1 %d", a.kseg1);
    return SFA_E_UNSUPPORTED;
  }
  if (epilogue == EPI_HEAD) {
    const int heads = a.N / 64;
    if (heads > SFA_MAX_HEADS) {
      set_error("conv: too many heads");
      return SFA_E_UNSUPPORTED;
    }
    if (a.M >= 256 * 256) return launch_cfg<256, 64, 64, 64, EPI_HEAD>(a, st);
    return launch_cfg<128, 64, 32, 64, EPI_HEAD>(a, st);
  }
  if (a.N % 128 == 0) {
    const long long big = (long long)ceil_div(a.M, 128) * (a.N / 128);
    if (big >= 512) return launch_cfg<128, 128, 64, 64, EPI_STD>(a, st);
    return launch_cfg<64, 128, 32, 64, EPI_STD>(a, st);
  }
  if ((long long)ceil_div(a.M, 256) * (a.N / 64) >= 512) return launch_cfg<256, 64, 64, 64, EPI_STD>(a, st);
  return launch_cfg<128, 64, 32, 64, EPI_STD>(a, st);
}

}  // namespace sfa
