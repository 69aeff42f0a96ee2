// Probe of gfx950's v_permlane16_swap / v_permlane32_swap (__builtin_amdgcn_permlane{16,32}_swap) and the DPP row
// controls (row_ror / mirrors) considered for csrc/kernels/common.h's lane reductions: prints, per lane, the two
// results of each swap with vdst = src = lane id, and the lane each DPP control reads.  Round 6 measured: swap32
// gives (l mod 32, l mod 32 + 32), swap16 the row pair, row_ror:n reads lane (l - n) mod 16 of the row.  (A
// __builtin_bit_cast of the swap builtin's vector element r[1] compiles to a read of element 0 — copy the elements
// to scalars first.)  Build: hipcc -O3 --offload-arch=gfx950 tools/probe/permlane_probe.hip -o /tmp/permlane_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned* out) {
  const unsigned l = threadIdx.x;
  const auto a = __builtin_amdgcn_permlane32_swap(l, l, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(l, l, false, false);
  const auto c = __builtin_amdgcn_permlane32_swap(l, l + 100, false, false);
  out[l * 10 + 0] = a[0];
  out[l * 10 + 1] = a[1];
  out[l * 10 + 2] = b[0];
  out[l * 10 + 3] = b[1];
  out[l * 10 + 4] = c[0];
  out[l * 10 + 5] = c[1];
  out[l * 10 + 6] = __builtin_amdgcn_update_dpp(0, (int)l, 0x124, 0xf, 0xf, false);
  out[l * 10 + 7] = __builtin_amdgcn_update_dpp(0, (int)l, 0x128, 0xf, 0xf, false);
  out[l * 10 + 8] = __builtin_amdgcn_update_dpp(0, (int)l, 0x141, 0xf, 0xf, false);
  out[l * 10 + 9] = __builtin_amdgcn_update_dpp(0, (int)l, 0x140, 0xf, 0xf, false);
}

int main() {
  unsigned* d;
  hipMalloc(&d, 640 * sizeof(unsigned));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  unsigned h[640];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("lane: swap32(l,l) | swap16(l,l) | swap32(l,l+100) | ror4 ror8 half_mirror mirror\n");
  for (int l = 0; l < 64; ++l)
    printf("%2d: %2u %2u | %2u %2u | %3u %3u | %2u %2u %2u %2u\n", l, h[l * 10], h[l * 10 + 1], h[l * 10 + 2],
           h[l * 10 + 3], h[l * 10 + 4], h[l * 10 + 5], h[l * 10 + 6], h[l * 10 + 7], h[l * 10 + 8], h[l * 10 + 9]);
  hipFree(d);
  return 0;
}
