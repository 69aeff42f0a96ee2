// Implicit-GEMM 3-D convolution on MFMA (gfx950): forward and dgrad.
//
// Layout: activations NDHWC bf16 (channels contiguous, arbitrary row stride so channel slices of a
// concatenated tensor are zero-copy views); weights packed K-contiguous [Ngemm][taps][C].
// One kernel template serves every conv class of SlowFast/Slow:
//   * k is ordered (tap, channel), so each 16-B (8 x bf16) or 8-B (4 x bf16, stems with RGB0 input)
//     chunk of a tile row is one contiguous global load of one tap; padding taps load zeros.
//   * A (gathered activations) and B (weights) are register-staged into a double-buffered LDS tile
//     (BK = 32, one MFMA k-step) with an XOR slot swizzle that makes every ds_read_b128 fragment read
//     conflict-free ((slot ^ ((row>>2)&1)<<1), brute-force checked against the b128 lane groups).
//   * Optional per-channel affine(+ReLU) is applied to A while staging: this is how a consumer conv
//     applies the producer's training-mode BatchNorm + ReLU without that activation ever being
//     materialised in HBM.
//   * The epilogue writes bf16 and (optionally) per-column partial sums (sum, sum of squares) of the
//     bf16-rounded output for the BatchNorm statistics: deterministic partial slabs, no atomics.
//   * MFMA operands are swapped (D = W·Xᵀ) so each lane ends up holding 4 consecutive channels of one
//     output position → one 8-B store per lane and a 16-lane shuffle for the channel sums.
//   * Linear workgroup ids go through the bijective XCD remap so the n-tiles of one m-tile share an L2.
#include "common.h"
#include "conv_params.h"
#include <type_traits>

namespace {

constexpr int BK = 32;

__device__ __forceinline__ int lds_off(int row, int slot) {
  // 64-byte rows (BK = 32 bf16), 16-byte slots.
  return row * 64 + ((slot ^ (((row >> 2) & 1) << 1)) << 4);
}

template <bool DGRAD>
__device__ __forceinline__ bool gather_coord(int base_c, int d, int s, int G, int& g) {
  if (!DGRAD) {
    g = base_c + d;
    return (unsigned)g < (unsigned)G;
  } else {
    int num = base_c - d;
    if (num < 0) return false;
    if (s == 1) { g = num; }
    else if (s == 2) { if (num & 1) return false; g = num >> 1; }
    else { int q = num / s; if (q * s != num) return false; g = q; }
    return g < G;
  }
}

template <int BM, int BN, int WM, int WN, int CH, bool DGRAD>
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64)
void conv_igemm_kernel(const ConvParams p) {
  constexpr int NWN = BN / WN;
  constexpr int NT = (BM / WM) * NWN * 64;
  constexpr int CPR = BK / CH;  // chunks per tile row
  constexpr int A_CHUNKS = BM * CPR, B_CHUNKS = BN * CPR;
  constexpr int A_SLOTS = (A_CHUNKS + NT - 1) / NT;
  constexpr int B_SLOTS = (B_CHUNKS + NT - 1) / NT;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int TILE_BYTES = (BM + BN) * BK * 2;
  static_assert(NT % CPR == 0, "thread count must be a multiple of chunks per row");
  using VT = typename std::conditional<CH == 8, uint4, uint2>::type;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem + 2 * TILE_BYTES);        // [2][BN] stats
  float* aff = red + 2 * BN;                                             // [2][Cg] affine

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / NWN, wn = wid % NWN;
  const int n_tiles = (p.Ngemm + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int tile_m = t / n_tiles, tile_n = t % n_tiles;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  const bool do_stats = p.stats != nullptr;
  const int affine = p.affine;
  if (do_stats) for (int i = tid; i < 2 * BN; i += NT) red[i] = 0.f;
  if (affine) {
    for (int i = tid; i < p.Cg; i += NT) { aff[i] = p.in_scale[i]; aff[p.Cg + i] = p.in_shift[i]; }
  }

  // ---- per-slot row coordinates (fixed over the K loop) ----
  const int col = tid % CPR;
  const int RHW = p.Rh * p.Rw, RTHW = p.Rt * RHW;
  const int GHW = p.Gh * p.Gw, GTHW = p.Gt * GHW;
  int a_base[A_SLOTS], a_t[A_SLOTS], a_h[A_SLOTS], a_w[A_SLOTS];
#pragma unroll
  for (int s = 0; s < A_SLOTS; ++s) {
    const int idx = tid + s * NT;
    const int m = m0 + idx / CPR;
    if (idx < A_CHUNKS && m < p.M) {
      const int b = m / RTHW;
      int r = m - b * RTHW;
      const int rt = r / RHW; r -= rt * RHW;
      const int rh = r / p.Rw; const int rw = r - rh * p.Rw;
      a_base[s] = b * GTHW;
      if (!DGRAD) { a_t[s] = rt * p.st - p.pt; a_h[s] = rh * p.sh - p.ph; a_w[s] = rw * p.sw - p.pw; }
      else        { a_t[s] = rt + p.pt;        a_h[s] = rh + p.ph;        a_w[s] = rw + p.pw; }
    } else {
      a_base[s] = 0; a_t[s] = -(1 << 28); a_h[s] = 0; a_w[s] = 0;
    }
  }

  // ---- k-state of this thread's column: (channel offset, tap) ----
  int kc = col * CH, kdt = 0, kdh = 0, kdw = 0;
  auto kadvance = [&](int by) {
    kc += by;
    while (kc >= p.Cg) {
      kc -= p.Cg;
      if (++kdw == p.kw) { kdw = 0; if (++kdh == p.kh) { kdh = 0; ++kdt; } }
    }
  };
  kadvance(0);

  VT ra[A_SLOTS], rb[B_SLOTS];
  int ra_c = 0;            // channel offset of the staged A chunks
  unsigned ra_valid = 0;   // bit s: slot s loaded real data
  int kglob = col * CH;    // k index of this thread's chunk in the current step

  auto load = [&]() {
    const bool tap_ok = kdt < p.kt;
    ra_c = kc; ra_valid = 0;
#pragma unroll
    for (int s = 0; s < A_SLOTS; ++s) {
      int gt, gh, gw;
      bool v = tap_ok && gather_coord<DGRAD>(a_t[s], kdt, p.st, p.Gt, gt) &&
               gather_coord<DGRAD>(a_h[s], kdh, p.sh, p.Gh, gh) &&
               gather_coord<DGRAD>(a_w[s], kdw, p.sw, p.Gw, gw);
      if (v) {
        const int64_t off = (int64_t)(a_base[s] + (gt * p.Gh + gh) * p.Gw + gw) * p.ldx + kc;
        ra[s] = *reinterpret_cast<const VT*>(p.x + off);
        ra_valid |= 1u << s;
      } else {
        ra[s] = VT{};
      }
    }
#pragma unroll
    for (int s = 0; s < B_SLOTS; ++s) {
      const int idx = tid + s * NT;
      const int n = n0 + idx / CPR;
      if (idx < B_CHUNKS && n < p.Ngemm && kglob < p.K)
        rb[s] = *reinterpret_cast<const VT*>(p.w + (int64_t)n * p.K + kglob);
      else
        rb[s] = VT{};
    }
    kadvance(BK);
    kglob += BK;
  };

  auto store_lds = [&](int buf) {
    char* A = smem + buf * TILE_BYTES;
    char* B = A + BM * BK * 2;
#pragma unroll
    for (int s = 0; s < A_SLOTS; ++s) {
      const int idx = tid + s * NT;
      if (idx >= A_CHUNKS) break;
      VT v = ra[s];
      if (affine && (ra_valid >> s & 1)) {
        float f[CH];
        if constexpr (CH == 8) unpack8(v, f); else unpack4(v, f);
#pragma unroll
        for (int e = 0; e < CH; ++e) {
          float z = f[e] * aff[ra_c + e] + aff[p.Cg + ra_c + e];
          f[e] = (affine == 2) ? fmaxf(z, 0.f) : z;
        }
        if constexpr (CH == 8) v = pack8(f); else v = pack4(f);
      }
      const int row = idx / CPR;
      if constexpr (CH == 8) *reinterpret_cast<VT*>(A + lds_off(row, col)) = v;
      else *reinterpret_cast<VT*>(A + lds_off(row, col >> 1) + (col & 1) * 8) = v;
    }
#pragma unroll
    for (int s = 0; s < B_SLOTS; ++s) {
      const int idx = tid + s * NT;
      if (idx >= B_CHUNKS) break;
      const int row = idx / CPR;
      if constexpr (CH == 8) *reinterpret_cast<VT*>(B + lds_off(row, col)) = rb[s];
      else *reinterpret_cast<VT*>(B + lds_off(row, col >> 1) + (col & 1) * 8) = rb[s];
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nsteps = (p.K + BK - 1) / BK;
  __syncthreads();  // affine table ready
  load();
  store_lds(0);
  __syncthreads();

  const int frow = lane & 15, fslot = lane >> 4;
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    const bool has_next = step + 1 < nsteps;
    if (has_next) load();
    const char* A = smem + cur * TILE_BYTES;
    const char* B = A + BM * BK * 2;
    bf16x8_t af[TM], bfr[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WM + i * 16 + frow;
      af[i] = *reinterpret_cast<const bf16x8_t*>(A + lds_off(row, fslot));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wn * WN + j * 16 + frow;
      bfr[j] = *reinterpret_cast<const bf16x8_t*>(B + lds_off(row, fslot));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    if (has_next) store_lds(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: D[n][m] fragment: lane holds channels n..n+3 of position m ----
  float cs[TN][4], cq[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { cs[j][r] = 0.f; cq[j][r] = 0.f; }

#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * WM + i * 16 + frow;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 16 + 4 * fslot;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (m < p.M && n < p.Ngemm) {
        uint16_t* dst = p.y + (int64_t)m * p.ldy + n;
        if (p.accum) {
          float o[4];
          unpack4(*reinterpret_cast<const uint2*>(dst), o);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += o[r];
        }
        const uint2 pk = pack4(v);
        *reinterpret_cast<uint2*>(dst) = pk;
        if (do_stats) {
          float q[4];
          unpack4(pk, q);
#pragma unroll
          for (int r = 0; r < 4; ++r) { cs[j][r] += q[r]; cq[j][r] += q[r] * q[r]; }
        }
      }
    }
  }
  if (do_stats) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s = sum16(cs[j][r]);
        const float q = sum16(cq[j][r]);
        if (frow == 0) {
          const int nl = wn * WN + j * 16 + 4 * fslot + r;
          atomicAdd(&red[nl], s);
          atomicAdd(&red[BN + nl], q);
        }
      }
    __syncthreads();
    for (int i = tid; i < BN; i += NT) {
      const int n = n0 + i;
      if (n < p.Ngemm) {
        p.stats[(int64_t)tile_m * 2 * p.Ngemm + n] = red[i];
        p.stats[(int64_t)tile_m * 2 * p.Ngemm + p.Ngemm + n] = red[BN + i];
      }
    }
  }
}

struct TileCfg { int bm, bn; };

template <int BM, int BN, int WM, int WN, int CH, bool DGRAD>
void launch_cfg(const ConvParams& p, hipStream_t stream) {
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  const int m_tiles = (p.M + BM - 1) / BM, n_tiles = (p.Ngemm + BN - 1) / BN;
  const size_t lds = 2 * (BM + BN) * BK * 2 + 2 * BN * 4 + (p.affine ? 2 * p.Cg * 4 : 0);
  hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, DGRAD>), dim3(m_tiles * n_tiles), dim3(NT), lds,
                     stream, p);
}

}  // namespace

// Tile selection by GEMM shape. Returns the BM used (callers size the stats slab with it).
int conv_igemm_pick_bm(int M, int N) {
  if (N > 64) {
    const long tiles = (long)((M + 127) / 128) * ((N + 127) / 128);
    return tiles >= 160 ? 128 : 128;
  }
  return N > 32 ? 128 : 256;
}

static int pick_variant(int M, int N) {
  if (N > 64) return 0;       // 128 x 128
  if (N > 32) return 1;       // 128 x 64
  if (N > 16) return 2;       // 256 x 32
  return 3;                   // 256 x 16
}

int conv_igemm_m_tiles(int M, int N) {
  const int v = pick_variant(M, N);
  const int bm = (v <= 1) ? 128 : 256;
  return (M + bm - 1) / bm;
}

void conv_igemm_launch(const ConvParams& p, int chunk, bool dgrad, hipStream_t stream) {
  const int v = pick_variant(p.M, p.Ngemm);
  if (dgrad) {
    switch (v) {
      case 0: launch_cfg<128, 128, 64, 64, 8, true>(p, stream); break;
      case 1: launch_cfg<128, 64, 64, 32, 8, true>(p, stream); break;
      case 2: launch_cfg<256, 32, 64, 32, 8, true>(p, stream); break;
      default: launch_cfg<256, 16, 64, 16, 8, true>(p, stream); break;
    }
  } else if (chunk == 8) {
    switch (v) {
      case 0: launch_cfg<128, 128, 64, 64, 8, false>(p, stream); break;
      case 1: launch_cfg<128, 64, 64, 32, 8, false>(p, stream); break;
      case 2: launch_cfg<256, 32, 64, 32, 8, false>(p, stream); break;
      default: launch_cfg<256, 16, 64, 16, 8, false>(p, stream); break;
    }
  } else {
    switch (v) {
      case 0: launch_cfg<128, 128, 64, 64, 4, false>(p, stream); break;
      case 1: launch_cfg<128, 64, 64, 32, 4, false>(p, stream); break;
      case 2: launch_cfg<256, 32, 64, 32, 4, false>(p, stream); break;
      default: launch_cfg<256, 16, 64, 16, 4, false>(p, stream); break;
    }
  }
}
