// Memory-bound helpers of the forward (HBM roofline; NHWC, float4 per lane).
//   nchw3_to_nhwc4      API input (B,3,H,W) -> (B,H,W,4)        test.py:124 boundary
//   maxpool3s2          fpn_resnet.py:123,182  MaxPool2d(3, 2, 1), -inf padding
//   upsample2x_bilinear fpn_resnet.py:198,202,207  F.interpolate(x2, bilinear, align_corners=True)
//   kfpn_combine        fpn_resnet.py:224-254  nearest-resize level 0, softmax over 3 levels,
//                       sum(v * softmax(v)), written NCHW per head
//   sigmoid_clamp       utils/torch_utils.py:44-45
#include "aux_kernels.h"

#include <algorithm>

#include "conv.h"

namespace sfa {

// FLIP: torch.flip(x, [H, W]) fused in (utils/demo_utils.py:110-111, the back view):
// pixel (h, w) of the output reads (H-1-h, W-1-w), i.e. flat index HW-1-p.
template <bool FLIP>
__global__ void __launch_bounds__(256) nchw3_to_nhwc4_kernel(const float* __restrict__ x,
                                                             float4* __restrict__ y, int HW,
                                                             unsigned* __restrict__ amax) {
  __shared__ float red[8];
  const int b = blockIdx.y;  // frame
  float mx = 0.f;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    const float* s = x + (size_t)b * 3 * HW + (FLIP ? HW - 1 - p : p);
    const float4 v = make_float4(s[0], s[HW], s[2 * HW], 0.f);
    y[(size_t)b * HW + p] = v;
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fabsf(v.z)));
  }
  if (amax) amax_commit_block<4>(amax, b, mx, 0.f, red);  // fp16x3 input scale (conv.h)
}

// Per-frame max |x| of an NHWC4 input handed to the forward as is (fp16x3 input scale).
__global__ void __launch_bounds__(256) amax_nhwc4_kernel(const float4* __restrict__ x, int HW,
                                                         unsigned* __restrict__ amax) {
  __shared__ float red[8];
  const int b = blockIdx.y;
  float mx = 0.f;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    const float4 v = x[(size_t)b * HW + p];
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  amax_commit_block<4>(amax, b, mx, 0.f, red);
}

// One thread per (output pixel, 4 channels) of one output row; grid (ceil(OW * C4 / 256), OH,
// B), 32-bit index math (C4 a power of two: no 64-bit divisions per thread).
__global__ void __launch_bounds__(256) maxpool3s2_kernel(const float4* __restrict__ x,
                                                         float4* __restrict__ y, int H, int W,
                                                         int logC4, int OH, int OW) {
  const int C4 = 1 << logC4;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= OW * C4) return;
  const int c = idx & (C4 - 1), ox = idx >> logC4, oy = blockIdx.y, b = blockIdx.z;
  const float4* xb = x + (size_t)b * H * W * C4;
  float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int iy = oy * 2 - 1 + dy;
    if ((unsigned)iy >= (unsigned)H) continue;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int ix = ox * 2 - 1 + dx;
      if ((unsigned)ix >= (unsigned)W) continue;
      const float4 v = xb[(iy * W + ix) * C4 + c];
      m.x = fmaxf(m.x, v.x);
      m.y = fmaxf(m.y, v.y);
      m.z = fmaxf(m.z, v.z);
      m.w = fmaxf(m.w, v.w);
    }
  }
  y[(((size_t)b * OH + oy) * OW + ox) * C4 + c] = m;
}

// align_corners=True: src = dst * (in-1)/(out-1) in f32 (ATen area_pixel_compute_scale /
// _source_index), i0 = floor(src), i1 = i0 + (i0 < in-1), l1 = src - i0, l0 = 1 - l1.
// Grid (ceil(OW * C4 / 256), OH, B) as maxpool3s2_kernel.
__device__ __forceinline__ float4 bilerp4(float ly0, float ly1, float lx0, float lx1, const float4& a00,
                                          const float4& a01, const float4& a10, const float4& a11) {
  float4 o;
  o.x = ly0 * (lx0 * a00.x + lx1 * a01.x) + ly1 * (lx0 * a10.x + lx1 * a11.x);
  o.y = ly0 * (lx0 * a00.y + lx1 * a01.y) + ly1 * (lx0 * a10.y + lx1 * a11.y);
  o.z = ly0 * (lx0 * a00.z + lx1 * a01.z) + ly1 * (lx0 * a10.z + lx1 * a11.z);
  o.w = ly0 * (lx0 * a00.w + lx1 * a01.w) + ly1 * (lx0 * a10.w + lx1 * a11.w);
  return o;
}

// Each thread owns one (output column, channel quad) over UP_ROWS consecutive output
// rows: with align_corners the source row advances by at most one per output row, so
// the two source rows stay in registers and are reloaded only when y0 moves (about
// 1.25 float4 loads per output instead of 4; 8 rows: -1..1.3 us per launch vs 4). Output rows are written in full 16-B quads
// along (ox, c): coalesced.
constexpr int UP_ROWS = 8;
__global__ void __launch_bounds__(256) upsample2x_bilinear_kernel(const float4* __restrict__ x,
                                                                  float4* __restrict__ y, int H,
                                                                  int W, int logC4, float sh,
                                                                  float sw) {
  const int C4 = 1 << logC4, OH = 2 * H, OW = 2 * W;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= OW * C4) return;
  const int c = idx & (C4 - 1), ox = idx >> logC4, b = blockIdx.z;
  const int oy0 = blockIdx.y * UP_ROWS;
  const float fx = sw * (float)ox;
  const int x0 = (int)fx;
  const int x1 = x0 + (x0 < W - 1 ? 1 : 0);
  const float lx1 = fx - (float)x0, lx0 = 1.f - lx1;
  const float4* xb = x + (size_t)b * H * W * C4;
  const int o0 = x0 * C4 + c, o1 = x1 * C4 + c, rs = W * C4;
  int cy0 = -1, cy1 = -1;
  float4 a00, a01, a10, a11;
  float4* yb = y + ((size_t)b * OH * OW + (size_t)oy0 * OW + ox) * C4 + c;
#pragma unroll
  for (int r = 0; r < UP_ROWS; ++r) {
    const int oy = oy0 + r;
    if (oy >= OH) break;
    const float fy = sh * (float)oy;
    const int y0 = (int)fy;
    const int y1 = y0 + (y0 < H - 1 ? 1 : 0);
    if (y0 != cy0) {
      if (y0 == cy1) {
        a00 = a10;
        a01 = a11;
      } else {
        a00 = xb[y0 * rs + o0];
        a01 = xb[y0 * rs + o1];
      }
      cy0 = y0;
    }
    if (y1 != cy1) {
      a10 = xb[y1 * rs + o0];
      a11 = xb[y1 * rs + o1];
      cy1 = y1;
    }
    const float ly1 = fy - (float)y0, ly0 = 1.f - ly1;
    yb[(size_t)r * OW * C4] = bilerp4(ly0, ly1, lx0, lx1, a00, a01, a10, a11);
  }
}

// Planar level buffers: Lk[ch][b][y][x] (ch over all heads, forward order).
// Level 0 is at (h/2, w/2) and resized by nearest (src = dst // 2, F.interpolate
// default mode with an exact 0.5 scale).
// grid (ceil(h * w / 4 / 256), B, channels), 4 pixels per thread: 32-bit index math.
__global__ void __launch_bounds__(256) kfpn_combine_kernel(const float* __restrict__ L0,
                                                           const float* __restrict__ L1,
                                                           const float* __restrict__ L2,
                                                           KfpnOut o, int B, int h, int w) {
  // every element by the same rounding sequence (no contraction), 4 consecutive pixels of a row
  // per thread (w % 4 == 0, checked at launch): float4 loads of levels 1 / 2 and of the output,
  // one float2 of level 0 (nearest: pixels 4q .. 4q + 3 read level-0 columns 2q, 2q + 1)
#pragma clang fp contract(off)
  const int hw = h * w;
  const int p = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (p >= hw) return;
  const int b = blockIdx.y, ch = blockIdx.z;
  const int yy = p / w, xx = p - yy * w;
  const int h0 = h / 2, w0 = w / 2;
  const float2 l0 = *reinterpret_cast<const float2*>(L0 + ((size_t)ch * B + b) * (h0 * w0) + (yy >> 1) * w0 + (xx >> 1));
  const float4 l1 = *reinterpret_cast<const float4*>(L1 + ((size_t)ch * B + b) * hw + p);
  const float4 l2 = *reinterpret_cast<const float4*>(L2 + ((size_t)ch * B + b) * hw + p);
  const float a0[4] = {l0.x, l0.x, l0.y, l0.y}, a1[4] = {l1.x, l1.y, l1.z, l1.w}, a2[4] = {l2.x, l2.y, l2.z, l2.w};
  float r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float v0 = a0[i], v1 = a1[i], v2 = a2[i];
    // softmax over the stacked last dim (torch: max-subtract, exp, sum, divide).
    const float mx = fmaxf(fmaxf(v0, v1), v2);
    const float e0 = expf(v0 - mx), e1 = expf(v1 - mx), e2 = expf(v2 - mx);
    const float sum = e0 + e1 + e2;
    const float w0_ = e0 / sum, w1_ = e1 / sum, w2_ = e2 / sum;
    r[i] = v0 * w0_ + v1 * w1_ + v2 * w2_;
  }
  // head of this channel
  int hd = 0;
#pragma unroll
  for (int j = 1; j < SFA_MAX_HEADS; ++j)
    if (j < o.num_heads && ch >= o.off[j]) hd = j;
  float* dst = o.ptr[0];
  int nc = o.ch[0];
#pragma unroll
  for (int j = 1; j < SFA_MAX_HEADS; ++j)
    if (j == hd) {
      dst = o.ptr[j];
      nc = o.ch[j];
    }
  const int c = ch - o.off[hd];
  *reinterpret_cast<float4*>(dst + ((size_t)b * nc + c) * hw + p) = make_float4(r[0], r[1], r[2], r[3]);
}

__global__ void __launch_bounds__(256) sigmoid_clamp_kernel(float* __restrict__ x, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float s = 1.0f / (1.0f + expf(-x[i]));
  x[i] = fminf(fmaxf(s, 1e-4f), 1.0f - 1e-4f);
}

static unsigned grid_of(long long n) { return (unsigned)((n + 255) / 256); }

// grid: (blocks per frame, frames); grid-stride within a frame keeps the amax commits few
static dim3 frame_grid(int B, long long HW) {
  return dim3((unsigned)std::min<long long>((HW + 255) / 256, 128), (unsigned)B);
}

int launch_nchw3_to_nhwc4(const float* x, float* y, int B, int H, int W, bool flip, unsigned* amax,
                          hipStream_t st) {
  if (B > 65535) {
    set_error("nchw3_to_nhwc4: batch %d too large", B);
    return SFA_E_INVALID;
  }
  if (flip)
    hipLaunchKernelGGL(nchw3_to_nhwc4_kernel<true>, frame_grid(B, (long long)H * W), dim3(256), 0, st,
                       x, reinterpret_cast<float4*>(y), H * W, amax);
  else
    hipLaunchKernelGGL(nchw3_to_nhwc4_kernel<false>, frame_grid(B, (long long)H * W), dim3(256), 0,
                       st, x, reinterpret_cast<float4*>(y), H * W, amax);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

int launch_amax_nhwc4(const float* x, int B, int H, int W, unsigned* amax, hipStream_t st) {
  if (B > 65535) {
    set_error("amax: batch %d too large", B);
    return SFA_E_INVALID;
  }
  hipLaunchKernelGGL(amax_nhwc4_kernel, frame_grid(B, (long long)H * W), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(x), H * W, amax);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

static int pow2_c4(int C, const char* what) {
  const int C4 = C / 4;
  if ((C & 3) || C4 <= 0 || (C4 & (C4 - 1))) {
    set_error("%s: channels %d must be 4 x a power of two", what, C);
    return -1;
  }
  return ilog2(C4);
}

int launch_maxpool3s2(const float* x, float* y, int B, int H, int W, int C, hipStream_t st) {
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int lc = pow2_c4(C, "maxpool3s2");
  if (lc < 0) return SFA_E_UNSUPPORTED;
  SFA_CHECK_ARG(B <= 65535 && OH <= 65535, "maxpool3s2: grid too large");
  hipLaunchKernelGGL(maxpool3s2_kernel, dim3((unsigned)((OW * (C / 4) + 255) / 256), (unsigned)OH, (unsigned)B),
                     dim3(256), 0, st, reinterpret_cast<const float4*>(x), reinterpret_cast<float4*>(y), H, W,
                     lc, OH, OW);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

int launch_upsample2x(const float* x, float* y, int B, int H, int W, int C, hipStream_t st) {
  const float sh = H > 1 ? (float)(H - 1) / (float)(2 * H - 1) : 0.f;
  const float sw = W > 1 ? (float)(W - 1) / (float)(2 * W - 1) : 0.f;
  const int lc = pow2_c4(C, "upsample2x");
  if (lc < 0) return SFA_E_UNSUPPORTED;
  SFA_CHECK_ARG(B <= 65535 && 2 * H <= 65535, "upsample2x: grid too large");
  hipLaunchKernelGGL(upsample2x_bilinear_kernel,
                     dim3((unsigned)((2 * W * (C / 4) + 255) / 256), (unsigned)((2 * H + UP_ROWS - 1) / UP_ROWS), (unsigned)B),
                     dim3(256), 0,
                     st, reinterpret_cast<const float4*>(x), reinterpret_cast<float4*>(y), H, W, lc, sh, sw);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

int launch_kfpn(const float* L0, const float* L1, const float* L2, const KfpnOut& o, int B, int h,
                int w, hipStream_t st) {
  SFA_CHECK_ARG(B <= 65535 && o.total_ch <= 65535, "kfpn: grid too large");
  SFA_CHECK_ARG(w % 4 == 0 && h % 2 == 0, "kfpn: head map %dx%d (width must be a multiple of 4)", h, w);
  hipLaunchKernelGGL(kfpn_combine_kernel, dim3((unsigned)((h * w / 4 + 255) / 256), (unsigned)B, (unsigned)o.total_ch),
                     dim3(256), 0, st, L0, L1, L2, o, B, h, w);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

__global__ void zero_words_kernel(uint4* __restrict__ p4, long long n4, unsigned* __restrict__ tail, int ntail) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) p4[i] = make_uint4(0u, 0u, 0u, 0u);
  if (i < ntail) tail[i] = 0u;
}

int launch_zero_words(void* p, size_t bytes, hipStream_t st) {
  if (bytes == 0) return SFA_OK;
  if (!p || (bytes & 3) || (reinterpret_cast<uintptr_t>(p) & 3)) {
    set_error("zero_words: %zu bytes at %p (need 4-B multiples, 4-B aligned)", bytes, p);
    return SFA_E_INVALID;
  }
  // 16-B stores up to the first 16-B boundary's multiple, words for the rest
  char* c = reinterpret_cast<char*>(p);
  const size_t head = (16 - (reinterpret_cast<uintptr_t>(c) & 15)) & 15;
  if (head >= bytes || bytes - head < 16) {
    const long long nw = (long long)(bytes / 4);
    hipLaunchKernelGGL(zero_words_kernel, dim3(grid_of(nw)), dim3(256), 0, st, nullptr, 0ll,
                       reinterpret_cast<unsigned*>(c), (int)nw);
    SFA_LAUNCH_CHECK();
    return SFA_OK;
  }
  const long long n4 = (long long)((bytes - head) / 16);
  if (head) {  // the few words before the 16-B boundary (one extra launch only for unaligned starts)
    hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(256), 0, st, nullptr, 0ll, reinterpret_cast<unsigned*>(c),
                       (int)(head / 4));
    SFA_LAUNCH_CHECK();
  }
  const size_t done = head + (size_t)n4 * 16;
  hipLaunchKernelGGL(zero_words_kernel, dim3(grid_of(n4 > 64 ? n4 : 64)), dim3(256), 0, st,
                     reinterpret_cast<uint4*>(c + head), n4, reinterpret_cast<unsigned*>(c + done),
                     (int)((bytes - done) / 4));
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

int launch_sigmoid_clamp(float* x, long long n, hipStream_t st) {
  if (n <= 0) return SFA_OK;
  hipLaunchKernelGGL(sigmoid_clamp_kernel, dim3(grid_of(n)), dim3(256), 0, st, x, n);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

}  // namespace sfa

extern "C" int sfa_sigmoid_clamp_inplace(float* x, int64_t n, void* stream) {
  SFA_CHECK_ARG(n >= 0 && (n == 0 || x), "sigmoid: bad arguments");
  return sfa::launch_sigmoid_clamp(x, n, reinterpret_cast<hipStream_t>(stream));
}
