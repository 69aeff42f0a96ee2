// GEMM-shaped microbenchmark of the implicit-GEMM conv kernel's big tiles (csrc/kernels/conv_igemm.hip), used to
// study their main-loop schedule in isolation: a dense 1x1 "conv" (x [M][K], packed w [N][K], y [M][N]) launched
// through the production template instances, bf16, timed with HIP events.  --hot 1 makes every row gather row 0
// (the A operand is L2-resident): the gap between hot and cold is what operand fetch costs the schedule.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I csrc/kernels tools/gemm_lab.hip -o build/gemm_lab
//   build/gemm_lab M N K [iters] [hot]
#define PVA_KERNEL_ONLY 1
#include "../csrc/kernels/conv_igemm.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <string>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace pva_bf16;

__global__ void fill_rand(uint16_t* p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    float f = ((h & 0xffff) / 65536.0f - 0.5f);
    p[i] = f2e(f);
  }
}

template <int BM, int BN, int WM, int WN, int BK, int UT>
float run(ConvParams p, int iters) {
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  const int m_tiles = (p.M + BM - 1) / BM, n_tiles = (p.Ngemm + BN - 1) / BN;
  const size_t lds = main_lds_bytes(BM, BN, BK, 0, dma_stages(BM, BN, BK, (UT & 17) == 17)) + (BM / WM) * 2 * BN * 4 +
                     ((UT & 32) ? (BM / WM) * (BN / WN) * 256 : 0);
  static_assert(!(UT & 64) || BK == 64, "interleaved schedule: BK=64 2-buffer loop");
  dim3 grid(m_tiles * n_tiles), block(NT);
  for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, 8, BK, 0, UT>), grid, block, lds, 0, p);
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, 8, BK, 0, UT>), grid, block, lds, 0, p);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGetLastError());
  return ms / iters;
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 250880, N = argc > 2 ? atoi(argv[2]) : 1024, K = argc > 3 ? atoi(argv[3]) : 1024;
  const int iters = argc > 4 ? atoi(argv[4]) : 20, hot = argc > 5 ? atoi(argv[5]) : 0;
  const std::string only = argc > 6 ? argv[6] : "";
  uint16_t *x, *w, *y;
  CK(hipMalloc(&x, (size_t)M * K * 2)); CK(hipMalloc(&w, (size_t)N * K * 2)); CK(hipMalloc(&y, (size_t)M * N * 2));
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, x, (size_t)M * K, 1u);
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, w, (size_t)N * K, 2u);
  ConvParams p{};
  p.x = x; p.w = w; p.y = y; p.M = M; p.Ngemm = N; p.Kfull = K; p.Cg = K; p.ldx = K; p.ldy = N;
  p.Gt = 1; p.Gh = 1; p.Gw = M; p.Rt = 1; p.Rh = 1; p.Rw = M; p.Ot = 1; p.Oh = 1; p.Ow = M;
  p.ost = p.osh = p.osw = 1; p.ast = p.ash = 1; p.asw = hot ? 0 : 1; p.dir = 1;
  p.nt = p.nh = p.nw = 1; p.kh = p.kw = 1; p.bts = p.bhs = p.bws = 1;
  p.xbytes = (unsigned)((size_t)M * K * 2); p.wbytes = (unsigned)((size_t)N * K * 2);
  const double flop = 2.0 * M * N * K;
  struct V { const char* name; float (*fn)(ConvParams, int); };
  std::vector<V> vs = {
      {"256x256/bk64/dma", run<256, 256, 128, 64, 64, 17>},
      {"256x256/bk32/dma", run<256, 256, 128, 64, 32, 17>},
      {"256x128/bk64/dma", run<256, 128, 128, 64, 64, 17>},
      {"256x128/bk32/dma", run<256, 128, 128, 64, 32, 17>},
      {"256x256/bk64/ut", run<256, 256, 128, 64, 64, 1>},
      {"256x256/bk64/dma/pf", run<256, 256, 128, 64, 64, 49>},
      {"256x256/bk32/dma/pf", run<256, 256, 128, 64, 32, 49>},
      {"256x128/bk64/dma/pf", run<256, 128, 128, 64, 64, 49>},
      {"256x128/bk32/dma/pf", run<256, 128, 128, 64, 32, 49>},
      {"256x256/bk64/dma/ilv", run<256, 256, 128, 64, 64, 81>},
      {"256x256/bk64/dma/pf/ilv", run<256, 256, 128, 64, 64, 113>},
      {"256x128/bk64/dma/pf/ilv", run<256, 128, 128, 64, 64, 113>},
  };
  for (auto& v : vs) {
    if (!only.empty() && only != v.name) continue;
    const float ms = v.fn(p, iters);
    printf("M=%d N=%d K=%d hot=%d %-20s %8.1f us %7.1f TF/s\n", M, N, K, hot, v.name, ms * 1e3, flop / ms / 1e9);
  }
  return 0;
}
