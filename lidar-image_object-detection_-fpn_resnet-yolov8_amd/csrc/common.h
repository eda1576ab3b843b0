// Shared helpers for the sfa_hip library (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/sfa_hip.h"

namespace sfa {

void set_error(const char* fmt, ...);

#define SFA_CHECK_ARG(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      ::sfa::set_error(__VA_ARGS__);        \
      return SFA_E_INVALID;                 \
    }                                       \
  } while (0)

#define SFA_HIP_TRY(expr)                                                                  \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) {                                                                \
      ::sfa::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                       __LINE__);                                                          \
      return SFA_E_HIP;                                                                    \
    }                                                                                      \
  } while (0)

// Checks the launch that was just enqueued (configuration errors only; no sync).
#define SFA_LAUNCH_CHECK()                                                                      \
  do {                                                                                          \
    hipError_t e_ = hipGetLastError();                                                          \
    if (e_ != hipSuccess) {                                                                     \
      ::sfa::set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(e_), __FILE__, \
                       __LINE__);                                                               \
      return SFA_E_HIP;                                                                         \
    }                                                                                           \
  } while (0)

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
inline int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

// CU count of the device a stream runs on (persistent-grid sizing), cached per device: each slot is
// written with the device's own answer, so concurrent first calls and launches on several devices
// agree; 256 (MI355X) when the query fails.
inline int cu_count(hipStream_t st) {
  constexpr int kMaxDev = 64;
  static std::atomic<int> cache[kMaxDev];
  int dev = -1;
  if (hipStreamGetDevice(st, &dev) != hipSuccess && hipGetDevice(&dev) != hipSuccess) return 256;
  if (dev < 0 || dev >= kMaxDev) return 256;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

// XCD-aware block remap (bijective for any grid size): blocks b and b+8 land
// on the same XCD under round-robin dispatch; give each XCD a contiguous chunk
// of logical tiles so neighbouring tiles share that XCD's L2.  Speed only.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int q = nblocks >> 3, r = nblocks & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace sfa
