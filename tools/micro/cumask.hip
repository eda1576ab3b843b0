// Which XCDs / CUs a stream's CU mask (hipExtStreamCreateWithCUMask) lets a kernel use: every
// block records its XCC id and CU id (s_getreg reads); a histogram per mask (tools only).
//   hipcc -O3 --offload-arch=gfx950 tools/micro/cumask.hip -o tools/micro/cumask
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>

__global__ void where(unsigned* out) {
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  // spin a little so the grid spreads over every allowed CU
  long long t0 = clock64();
  while (clock64() - t0 < 20000) {}
  if (threadIdx.x == 0) out[blockIdx.x] = (xcc & 0xf) << 16 | (hw & 0xffff);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int nw = (ncu + 31) / 32, nb = 4096;
  unsigned* d;
  hipMalloc(&d, nb * 4);
  std::vector<unsigned> h(nb);
  const char* names[] = {"all", "cu 0..127", "cu 128..255", "even cu", "cu%8<4", "cu%64<32"};
  for (int v = 0; v < 6; ++v) {
    std::vector<unsigned> m(nw, 0u);
    for (int c = 0; c < ncu; ++c) {
      bool on = v == 0 || (v == 1 && c < ncu / 2) || (v == 2 && c >= ncu / 2) || (v == 3 && c % 2 == 0) ||
                (v == 4 && c % 8 < 4) || (v == 5 && c % 64 < 32);
      if (on) m[c / 32] |= 1u << (c % 32);
    }
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, nw, m.data()) != hipSuccess) { printf("%s: create failed\n", names[v]); continue; }
    hipMemset(d, 0xff, nb * 4);
    hipLaunchKernelGGL(where, dim3(nb), dim3(64), 0, s, d);
    hipStreamSynchronize(s);
    hipMemcpy(h.data(), d, nb * 4, hipMemcpyDeviceToHost);
    int xcd[16] = {0};
    std::vector<int> cus;
    for (unsigned w : h) {
      xcd[(w >> 16) & 15]++;
      unsigned key = w;  // (xcc, hw id) pairs -> distinct CUs
      bool seen = false;
      for (int c : cus) if ((unsigned)c == (key & 0xfff00f0fu)) { seen = true; break; }
      if (!seen) cus.push_back((int)(key & 0xfff00f0fu));
    }
    printf("%-12s blocks per XCC:", names[v]);
    for (int x = 0; x < 8; ++x) printf(" %5d", xcd[x]);
    printf("   distinct (xcc, se, cu) ~%zu\n", cus.size());
    hipStreamDestroy(s);
  }
  return 0;
}
