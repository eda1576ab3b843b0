// Convolution dispatch: picks the conv_mfma_kernel tile configuration per layer
// shape (see conv_kernel.h for the kernel; DESIGN.md §5 for the rooflines).
#include "conv_kernel.h"

namespace sfa {

int launch_conv(const ConvArgs& a, int epilogue, hipStream_t st) {
  // Host-side shape checks: the kernels assume these and never bounds-check them.
  if (a.N <= 0 || a.N % 64 != 0 || a.M <= 0 || a.Kpad <= 0 || a.Kpad % 16 != 0) {
    set_error("conv: unsupported shape M=%d N=%d Kpad=%d", a.M, a.N, a.Kpad);
    return SFA_E_UNSUPPORTED;
  }
  for (int s = 0; s < a.nseg; ++s) {
    const ConvSeg& g = a.seg[s];
    if (!g.x || g.C < 4 || (g.C & (g.C - 1)) || (1 << g.logC) != g.C || g.KW <= 0 || g.KH <= 0) {
      set_error("conv: bad segment %d (C=%d)", s, g.C);
      return SFA_E_UNSUPPORTED;
    }
    if (g.bytes == 0 || g.bytes >= (1u << 31)) {
      set_error("conv: segment %d input is empty or >= 2 GiB (32-bit buffer offsets)", s);
      return SFA_E_UNSUPPORTED;
    }
    if (g.C < 16 && s != a.nseg - 1) {
      set_error("conv: narrow-channel segment must be last");
      return SFA_E_UNSUPPORTED;
    }
  }
  if (a.nseg == 2 && (a.kseg1 % 16 != 0 || a.kseg1 <= 0 || a.kseg1 >= a.Kpad)) {
    set_error("conv: bad kseg1 %d", a.kseg1);
    return SFA_E_UNSUPPORTED;
  }
  // Tile choice per shape, from tools/convbench.hip sweeps on MI355X (round 1):
  // 32x64 / 32x32 wave tiles at 4 waves per SIMD hide the gather latency best;
  // BK = 32 pays only for the long-K, few-block layer4 shapes; the LDS-DMA ring
  // (GLDS) gains 2-8 % on the heads and layer3, nothing elsewhere.
  if (epilogue == EPI_HEAD) {
    if (a.N / 64 > SFA_MAX_HEADS) {
      set_error("conv: too many heads");
      return SFA_E_UNSUPPORTED;
    }
    return launch_conv_cfg<128, 64, 32, 64, 16, EPI_HEAD, 4, true>(a, st);
  }
  if (a.N == 64) return launch_conv_cfg<128, 64, 32, 64, 16, EPI_STD, 4>(a, st);
  if (a.N % 128 == 0) {
    if ((long long)ceil_div(a.M, 128) * (a.N / 128) >= 512)
      return launch_conv_cfg<128, 128, 64, 64, 16, EPI_STD, 3>(a, st);
    if ((long long)ceil_div(a.M, 64) * (a.N / 128) >= 512)
      return launch_conv_cfg<64, 128, 32, 64, 16, EPI_STD, 4, true>(a, st);
    if (a.Kpad % 32 == 0 && (a.nseg == 1 || a.kseg1 % 32 == 0))
      return launch_conv_cfg<64, 64, 32, 32, 32, EPI_STD, 4>(a, st);
  }
  return launch_conv_cfg<64, 64, 32, 32, 16, EPI_STD, 4>(a, st);
}

}  // namespace sfa
