// Halo-staged implicit-GEMM forward and dgrad of stride-1 'same' (1,3,3) convolutions on MFMA (gfx950):
// the spatial conv_b of every bottleneck whose output rows are the input rows (SlowFast slow res2-res4).
//
//   y[p][n] = sum_{tap, c} x'[p + off(tap)][c] * w[n][tap][c]        (x' = BN+ReLU(x) recomputed, or x)
//
// The tile kernel of conv_igemm.hip gathers one im2col row per (position, tap): each activation is fetched
// from L2 and put through the consumer-side BN+ReLU nine times, and at 64-128 channels that L2 traffic
// (~1.2 KB per output position at K = 576) bounds the GEMM well below the matrix cores (slow res2 conv_b ran
// at ~420 TF/s).  Here a workgroup owns R full image rows x all W columns of one frame (P = R*W <= 224
// positions) and an n-tile of 64 or 128 output channels:
//   * the input HALO [(R+2) x (W+2)][CK channels] is staged into LDS ONCE (global -> registers -> BN+ReLU ->
//     ds_write; padding positions are zeros, so no bounds test in the MFMA loop), in slices of CK <= 128
//     channels;
//   * LDS image is channel-group-major: [CK/8][positions padded to 16][8 bf16], so the 16 positions x 4
//     channel groups of one ds_read_b128 fragment land on 16 distinct 16-B bank groups (position p of group g
//     at unit (g*NPOSP + p) mod 16 with NPOSP = 0 mod 16) with no XOR swizzle, and every tap of a fragment is
//     the same per-lane address plus a wave-uniform offset (dh*(W+2) + dw)*16;
//   * the weight fragments are read straight from global memory into registers (16 B per lane, L2-resident,
//     prefetched 2 (128-channel tiles) or 5 (64-channel tiles) k-steps ahead), so the k loop has no barrier at all;
//   * 4 waves = 2 position halves x 2 channel halves, each wave up to 7 x (NTILE/32) 16x16 accumulators;
//     v_mfma_f32_16x16x32_bf16 with swapped operands (D = W X^T) so each lane holds 4 consecutive channels of
//     one position (8-B stores, 16-lane shuffles for the channel sums), exactly like conv_igemm.hip;
//   * epilogues: EPI 0 = raw output + BN partial sums [tiles][2][N] (sum, sum of squares of the bf16 output);
//     EPI 1 = the dgrad epilogue of a conv whose input is relu(BN_a(y0)): ReLU mask recomputed from y0,
//     masked gradient stored, BN_a backward partials [tiles][3][N] (sum v, sum v*xhat0, 0).
// Launch word (conv_igemm_launch): bit 4 explicit, bit 11 this kernel, bit 0 = 64-channel n-tiles (else 128),
// bits 12+ = positions per tile P (so conv_cfg_bm = P and the partial-sum tile count is M / P).
#include "common.h"
#include "conv_params.h"

PVA_NS_BEGIN

namespace {

constexpr int HC_THREADS = 256;
constexpr int HC_MW = 7;        // 16-position blocks per wave (two position halves of <= 112)
constexpr int HC_PMAX = 2 * HC_MW * 16;
// weight-fragment ring depth (k-steps in flight): a 64-channel tile's k-step is only 14 MFMAs per wave, so it keeps
// five steps of L2 latency in flight; a 128-channel tile's 28-MFMA steps need two
__host__ __device__ constexpr int hc_ring(int ntile) { return ntile == 64 ? 6 : 3; }

// rows per tile: the largest divisor R of H with R*W <= 224 (every tile is whole rows of one frame)
__host__ __device__ inline int halo_rows(int H, int W) {
  for (int r = H; r >= 1; --r)
    if (H % r == 0 && r * W <= HC_PMAX) return r;
  return 0;
}

__host__ __device__ inline int halo_ck(int Cg) { return Cg <= 128 ? Cg : 128; }

template <int NTILE, int EPI, int AFF>
__global__ __launch_bounds__(HC_THREADS, 2) void conv_halo_kernel(const ConvParams p, const int R) {
  constexpr int NWB = NTILE / 32;   // 16-channel blocks per wave
  constexpr int HC_RING = hc_ring(NTILE);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid & 1, wn = wid >> 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int W = p.Rw, H = p.Rh;
  const int PW = W + 2;
  const int P = R * W;
  const int NPOS = (R + 2) * PW, NPOSP = (NPOS + 15) & ~15;
  const int CK = halo_ck(p.Cg);
  const int G8 = CK >> 3;
  const int box_bytes = G8 * NPOSP * 16;
  float* red = reinterpret_cast<float*>(smem + box_bytes);    // [2 halves][2 or 3][NTILE]
  float* aff = red + (EPI ? 6 : 4) * NTILE;                   // [2][Cg] consumer-side affine
  float* bnp = aff + (AFF ? 2 * p.Cg : 0);                    // EPI 1: [4][NTILE] mean0 rstd0 msc msh

  const int n_tiles = (p.Ngemm + NTILE - 1) / NTILE;
  const int t = xcd_remap(blockIdx.x, gridDim.x);   // the n-tiles of one m-tile (same halo) share an XCD
  const int tile_m = t / n_tiles, tile_n = t - (t / n_tiles) * n_tiles;
  const int tpf = H / R;
  const int frame = tile_m / tpf, r0 = (tile_m - frame * tpf) * R;
  const int n0 = tile_n * NTILE;
  const int fbase = frame * H * W;   // first row of this frame (gathered and output tensors share the grid)

  if constexpr (AFF != 0) {
    for (int i = tid; i < p.Cg; i += HC_THREADS) { aff[i] = p.in_scale[i]; aff[p.Cg + i] = p.in_shift[i]; }
  }
  if constexpr (EPI == 1) {
    for (int i = tid; i < NTILE; i += HC_THREADS) {
      const int n = min(n0 + i, p.Ngemm - 1);
      bnp[i] = p.emean0[n]; bnp[NTILE + i] = p.erstd0[n];
      bnp[2 * NTILE + i] = p.emsc[n]; bnp[3 * NTILE + i] = p.emsh[n];
    }
  }

  // ---- per-lane fragment addresses
  const int mwr = min(HC_MW, ((P + 15) / 16 + 1) / 2);   // live 16-position blocks per wave
  int abase[HC_MW];
#pragma unroll
  for (int i = 0; i < HC_MW; ++i) {
    const int pl = min((wm * mwr + i) * 16 + fr, P - 1);
    const int h = pl / W, w = pl - h * W;
    abase[i] = (fg * NPOSP + (h + 1) * PW + (w + 1)) * 16;
  }
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)p.wbytes, 0x00020000);
  int bvo[NWB];
#pragma unroll
  for (int j = 0; j < NWB; ++j) {
    const int n = min(n0 + wn * (NTILE / 2) + j * 16 + fr, p.Ngemm - 1);
    bvo[j] = (n * p.Kfull + fg * 8) * 2;
  }
  // k-steps: (slice c, tap, 32-channel step kc); taps in (jh, jw) order
  const int ksl = CK / 32;
  const int nsteps = (p.Cg / 32) * 9;
  auto step_w = [&](int s) {   // byte offset of step s in a packed weight row
    const int c = s / (9 * ksl);
    const int r = s - c * 9 * ksl;
    const int tap = r / ksl, kc = r - tap * ksl;
    const int jh = tap / 3, jw = tap - jh * 3;
    const int wt = (p.bt0 * p.kh + p.bh0 + jh * p.bhs) * p.kw + p.bw0 + jw * p.bws;
    return (wt * p.Cg + c * CK + kc * 32) * 2;
  };
  auto step_a = [&](int s) {   // uniform byte offset of step s in the halo image
    const int c = s / (9 * ksl);
    const int r = s - c * 9 * ksl;
    const int tap = r / ksl, kc = r - tap * ksl;
    const int jh = tap / 3, jw = tap - jh * 3;
    const int dh = p.aoh + p.dir * jh, dw = p.aow + p.dir * jw;
    return (dh * PW + dw + kc * 4 * NPOSP) * 16;
  };

  f32x4_t acc[HC_MW][NWB];
#pragma unroll
  for (int i = 0; i < HC_MW; ++i)
#pragma unroll
    for (int j = 0; j < NWB; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint4 bq[HC_RING][NWB];
  auto bload = [&](int s, uint4 (&dst)[NWB]) {
    const int so = step_w(min(s, nsteps - 1));
#pragma unroll
    for (int j = 0; j < NWB; ++j)
      dst[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wr, bvo[j], so, 0));
  };
#pragma unroll
  for (int u = 0; u < HC_RING - 1; ++u) bload(u, bq[u]);

  // ---- halo staging: thread -> (channel group cg, 8 consecutive box positions per pass-row)
  const int cg = (tid >> 3) % G8;
  const int ppp = HC_THREADS / G8;                  // box positions per pass
  const int b_first = ((tid >> 3) / G8) * 8 + (tid & 7);
  auto stage = [&](int c) {
    float sc[8], sh[8];
    if constexpr (AFF != 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { sc[e] = aff[c * CK + cg * 8 + e]; sh[e] = aff[p.Cg + c * CK + cg * 8 + e]; }
    }
    const int coff = c * CK + cg * 8;
    int hh = b_first / PW, ww = b_first - (b_first / PW) * PW;
    constexpr int BATCH = 6;
    for (int b0 = b_first; b0 < NPOS; b0 += BATCH * ppp) {
      uint4 v[BATCH];
      bool ok[BATCH];
      int bb[BATCH];
#pragma unroll
      for (int u = 0; u < BATCH; ++u) {
        const int b = b0 + u * ppp;
        bb[u] = b;
        const int h = r0 - 1 + hh, w = ww - 1;
        ok[u] = b < NPOS && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        v[u] = uint4{0, 0, 0, 0};
        if (ok[u]) v[u] = *reinterpret_cast<const uint4*>(p.x + (size_t)(fbase + h * W + w) * p.ldx + coff);
        ww += ppp;
        while (ww >= PW) { ww -= PW; ++hh; }
      }
#pragma unroll
      for (int u = 0; u < BATCH; ++u) {
        if (bb[u] >= NPOS) break;
        uint4 o = v[u];
        if constexpr (AFF != 0) {
          float f[8];
          unpack8(o, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = __builtin_fmaf(f[e], sc[e], sh[e]);
          o = pack8_fast(f);
          if constexpr (AFF == 2) o = relu_e16x8(o);
          if (!ok[u]) o = uint4{0, 0, 0, 0};   // zero padding of the activation itself
        }
        *reinterpret_cast<uint4*>(smem + (cg * NPOSP + bb[u]) * 16) = o;
      }
    }
  };

  __syncthreads();   // affine / BN tables
  const int nslices = p.Cg / CK;
  int s = 0;
  for (int c = 0; c < nslices; ++c) {
    if (c > 0) __syncthreads();   // every wave is done with the previous slice
    stage(c);
    __syncthreads();
    const int send = s + 9 * ksl;
    // HC_RING k-steps per iteration: the weight ring slot of each is compile-time
    for (; s < send; s += HC_RING) {
#pragma unroll
      for (int u = 0; u < HC_RING; ++u) {
        const int ss = s + u;
        bload(ss + HC_RING - 1, bq[(u + HC_RING - 1) % HC_RING]);
        const int ao = step_a(ss);
        ev8_t af[HC_MW];
#pragma unroll
        for (int i = 0; i < HC_MW; ++i)
          if (i < mwr) af[i] = *reinterpret_cast<const ev8_t*>(smem + abase[i] + ao);
#pragma unroll
        for (int i = 0; i < HC_MW; ++i) {
          if (i >= mwr) continue;
#pragma unroll
          for (int j = 0; j < NWB; ++j)
            acc[i][j] = PVA_MFMA16(__builtin_bit_cast(ev8_t, bq[u][j]), af[i],
                                                                acc[i][j], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue
  const int ncol0 = wn * (NTILE / 2);
  if constexpr (EPI == 0) {
    const bool do_stats = p.stats != nullptr;
    float cs[NWB][4], cq[NWB][4];
#pragma unroll
    for (int j = 0; j < NWB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) { cs[j][r] = 0.f; cq[j][r] = 0.f; }
#pragma unroll
    for (int i = 0; i < HC_MW; ++i) {
      if (i >= mwr) continue;
      const int pl = (wm * mwr + i) * 16 + fr;
      if (pl >= P) continue;
      const int row = fbase + r0 * W + pl;
#pragma unroll
      for (int j = 0; j < NWB; ++j) {
        const int n = n0 + ncol0 + j * 16 + 4 * fg;
        if (n >= p.Ngemm) continue;
        const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        const uint2 pk = pack4(v);
        *reinterpret_cast<uint2*>(p.y + (size_t)row * p.ldy + n) = pk;
        if (do_stats) {
          float q[4];
          unpack4(pk, q);
#pragma unroll
          for (int r = 0; r < 4; ++r) { cs[j][r] += q[r]; cq[j][r] += q[r] * q[r]; }
        }
      }
    }
    if (!do_stats) return;
#pragma unroll
    for (int j = 0; j < NWB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = sum16(cs[j][r]), b = sum16(cq[j][r]);
        if (fr == 0) {
          const int nl = ncol0 + j * 16 + 4 * fg + r;
          red[(wm * 2) * NTILE + nl] = a;
          red[(wm * 2 + 1) * NTILE + nl] = b;
        }
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int i = tid; i < NTILE; i += HC_THREADS) {
      const int n = n0 + i;
      if (n < p.Ngemm) {
        p.stats[(tile_m * 2) * p.Ngemm + n] = red[i] + red[2 * NTILE + i];
        p.stats[(tile_m * 2 + 1) * p.Ngemm + n] = red[NTILE + i] + red[3 * NTILE + i];
      }
    }
  } else {
    // dgrad of a conv whose input is relu(BN_a(y0)): v = acc * (y0*msc + msh > 0); sums v, v*y0
    float sv[NWB][4], s0[NWB][4];
#pragma unroll
    for (int j = 0; j < NWB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) { sv[j][r] = 0.f; s0[j][r] = 0.f; }
#pragma unroll
    for (int i = 0; i < HC_MW; ++i) {
      if (i >= mwr) continue;
      const int pl = (wm * mwr + i) * 16 + fr;
      if (pl >= P) continue;
      const int row = fbase + r0 * W + pl;
#pragma unroll
      for (int j = 0; j < NWB; ++j) {
        const int nl = ncol0 + j * 16 + 4 * fg;
        const int n = n0 + nl;
        if (n >= p.Ngemm) continue;
        float a[4];
        unpack4(*reinterpret_cast<const uint2*>(p.ey0 + (size_t)row * p.Ngemm + n), a);
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
          v[r] = (a[r] * bnp[2 * NTILE + nl + r] + bnp[3 * NTILE + nl + r] > 0.f) ? acc[i][j][r] : 0.f;
        const uint2 pk = pack4(v);
        *reinterpret_cast<uint2*>(p.y + (size_t)row * p.ldy + n) = pk;
        float q[4];
        unpack4(pk, q);
#pragma unroll
        for (int r = 0; r < 4; ++r) { sv[j][r] += q[r]; s0[j][r] += q[r] * a[r]; }
      }
    }
#pragma unroll
    for (int j = 0; j < NWB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nl = ncol0 + j * 16 + 4 * fg + r;
        const float a = sum16(sv[j][r]), b = sum16(s0[j][r]);
        if (fr == 0) {
          red[(wm * 3) * NTILE + nl] = a;
          red[(wm * 3 + 1) * NTILE + nl] = (b - bnp[nl] * a) * bnp[NTILE + nl];   // sum v*xhat0
        }
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int i = tid; i < NTILE; i += HC_THREADS) {
      const int n = n0 + i;
      if (n < p.Ngemm) {
        p.epart[(tile_m * 3) * p.Ngemm + n] = red[i] + red[3 * NTILE + i];
        p.epart[(tile_m * 3 + 1) * p.Ngemm + n] = red[NTILE + i] + red[4 * NTILE + i];
        p.epart[(tile_m * 3 + 2) * p.Ngemm + n] = 0.f;
      }
    }
  }
}

template <int NTILE, int EPI, int AFF>
void launch_one(const ConvParams& p, int R, hipStream_t st) {
  const int W = p.Rw;
  const int NPOSP = (((R + 2) * (W + 2)) + 15) & ~15;
  const int CK = halo_ck(p.Cg);
  const size_t lds = (size_t)(CK / 8) * NPOSP * 16 + (EPI ? 6 : 4) * NTILE * 4 + (AFF ? 2 * p.Cg * 4 : 0) +
                     (EPI ? 4 * NTILE * 4 : 0);
  const int m_tiles = p.M / (R * W);
  const int n_tiles = (p.Ngemm + NTILE - 1) / NTILE;
  hipLaunchKernelGGL((conv_halo_kernel<NTILE, EPI, AFF>), dim3(m_tiles * n_tiles), dim3(HC_THREADS), lds, st, p, R);
}

template <int NTILE>
void launch_ntile(const ConvParams& p, int R, bool epi, hipStream_t st) {
  if (epi) { launch_one<NTILE, 1, 0>(p, R, st); return; }
  switch (p.affine) {
    case 0: launch_one<NTILE, 0, 0>(p, R, st); break;
    case 1: launch_one<NTILE, 0, 1>(p, R, st); break;
    default: launch_one<NTILE, 0, 2>(p, R, st); break;
  }
}


// ------------------------------------------------------------------------------------------------------------------
// Persistent 64 -> 64 channel variant (slow res2 conv_b, 56x56: the kernel above runs it at ~17 % MFMA busy, waits
// 0.37, profiles/r3_pmc/halo_bench_pmc.txt).  What changes:
//   * the whole weight tensor (64 x 9 x 64 bf16 = 72 KB) is staged into LDS ONCE per workgroup, in k-step-major,
//     channel-group-major order [18 k-steps][4 groups][64 n][8] (a fragment's 16 lanes of one group hit 16 distinct
//     16-B bank slots), instead of re-fetching weight fragments from L2 every k-step;
//   * one workgroup of 8 waves per CU walks a contiguous range of tiles (R x W positions of one frame, P <= 224):
//     the next tile's halo is loaded into registers (6 x 16 B per lane, one 128-B position row per 8 lanes) while
//     the current tile computes, and written to LDS (BN+ReLU applied) behind one barrier;
//   * compile-time channel counts: no runtime divisions in the k loop (18 fully unrolled k-steps, per-tap halo
//     offsets in SGPRs), 8 waves = 2 channel halves (2 x 16-channel blocks) x 4 position groups (3-4 blocks of 16).
// Epilogues as conv_halo_kernel (EPI 0: raw output + BN partial sums per tile; EPI 1: dgrad with the BN_a ReLU mask
// from y0 and the BN_a backward partials).  LDS: 72 KB weights + 8 x NPOSP x 16 B halo (<= 44 KB) + reductions.
constexpr int HP_THREADS = 512;
constexpr int HP_NPOSP_MAX = 352;   // (R + 2) x (W + 2) halo positions, padded to 16
constexpr int HP_STG = (HP_NPOSP_MAX * 8 + HP_THREADS - 1) / HP_THREADS;   // 16-B halo chunks per thread

__host__ __device__ inline int hp_nposp(int R, int W) { return (((R + 2) * (W + 2)) + 15) & ~15; }

// DIR = +1 (forward, tap offsets -1..1) or -1 (dgrad, flipped taps); WW x RR = image width x rows per tile: every
// halo offset is a compile-time constant folded into the ds_read immediates (runtime offsets were hoisted out of the
// tile loop by the compiler into ~70 address VGPRs and spilled)
template <int EPI, int AFF, int DIR, int WW, int RR>
__global__ __launch_bounds__(HP_THREADS, 1) void conv_halo64p_kernel(const ConvParams p, const int ntiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int C = 64;
  constexpr int W = WW, R = RR;
  constexpr int PW = W + 2;
  constexpr int P = R * W;
  constexpr int NPOS = (R + 2) * PW, NPOSP = (NPOS + 15) & ~15;
  static_assert(NPOSP <= HP_NPOSP_MAX && P <= 224, "halo tile too large");
  char* WI = smem;                                   // [18][4][64][16 B] weights
  char* HI = smem + 18 * 4 * 64 * 16;                // [8][NPOSP][16 B] halo
  const int H = p.Rh;
  float* red = reinterpret_cast<float*>(HI + 8 * NPOSP * 16);   // [4 wm][3][64]
  float* bnp = red + 4 * 3 * C;                                 // EPI 1: [4][64] mean0 rstd0 msc msh; then aff

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid & 1, wm = wid >> 1;
  const int fr = lane & 15, fg = lane >> 4;
  // contiguous tile range of this workgroup (neighbouring tiles share halo rows through this XCD's L2)
  const int t_begin = (int)((long long)blockIdx.x * ntiles / gridDim.x);
  const int t_end = (int)((long long)(blockIdx.x + 1) * ntiles / gridDim.x);
  const int tpf = H / R;

  // ---- per-tap uniform offsets (the geometry of conv_halo_kernel's step_w / step_a with one 64-channel slice)
  int wtap[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int jh = tap / 3, jw = tap - jh * 3;
    wtap[tap] = (p.bt0 * p.kh + p.bh0 + jh * p.bhs) * p.kw + p.bw0 + jw * p.bws;
  }
  // ---- weights -> LDS: chunk q = (s, g, n): k-step s = 2 tap + half, channel group g, output channel n
  for (int q = tid; q < 18 * 4 * 64; q += HP_THREADS) {
    const int s = q >> 8, g = (q >> 6) & 3, n = q & 63;
    const int tap = s >> 1, half = s & 1;
    int wt = 0;
#pragma unroll
    for (int u = 0; u < 9; ++u) wt = (u == tap) ? wtap[u] : wt;
    *reinterpret_cast<uint4*>(WI + q * 16) =
        *reinterpret_cast<const uint4*>(p.w + (size_t)n * p.Kfull + wt * C + half * 32 + g * 8);
  }
  if constexpr (EPI == 1) {
    for (int i = tid; i < C; i += HP_THREADS) {
      bnp[i] = p.emean0[i]; bnp[C + i] = p.erstd0[i]; bnp[2 * C + i] = p.emsc[i]; bnp[3 * C + i] = p.emsh[i];
    }
  }

  // ---- staging roles: lane -> channel group cg = lane >> 3, position u*64 + wid*8 + (lane & 7) of pass u
  const int cg = lane >> 3;
  float* aff = bnp + 4 * C;   // [2][64] consumer-side affine (read per tile from LDS: fewer live VGPRs)
  if constexpr (AFF != 0) {
    for (int i = tid; i < C; i += HP_THREADS) { aff[i] = p.in_scale[i]; aff[C + i] = p.in_shift[i]; }
  }
  // per pass: halo row hh (bits 16-23), column-in-image flag (bit 24), row offset (h-1)*W + (w-1) + 2^15 (bits 0-15)
  int hcode[HP_STG];
#pragma unroll
  for (int u = 0; u < HP_STG; ++u) {
    const int pos = u * 64 + wid * 8 + (lane & 7);
    const int h = pos / PW, w = pos - h * PW;
    const bool ok = pos < NPOS && w >= 1 && w <= W;
    hcode[u] = ok ? ((h << 16) | (1 << 24) | ((h - 1) * W + (w - 1) + 32768)) : 0;
  }
  auto load_halo = [&](int t, uint4 (&stg)[HP_STG]) {
    const int frame = t / tpf, r0 = (t - frame * tpf) * R;
    const uint16_t* base = p.x + ((size_t)frame * H * W + (size_t)r0 * W) * p.ldx + cg * 8;
#pragma unroll
    for (int u = 0; u < HP_STG; ++u) {
      const int h = r0 - 1 + ((hcode[u] >> 16) & 255);
      stg[u] = uint4{0, 0, 0, 0};
      if ((hcode[u] >> 24) && (unsigned)h < (unsigned)H)
        stg[u] = *reinterpret_cast<const uint4*>(base + (ptrdiff_t)((hcode[u] & 65535) - 32768) * p.ldx);
    }
  };
  auto store_halo = [&](int t, const uint4 (&stg)[HP_STG]) {
    const int frame = t / tpf, r0 = (t - frame * tpf) * R;
    float sc[8], sh[8];
    if constexpr (AFF != 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { sc[e] = aff[cg * 8 + e]; sh[e] = aff[C + cg * 8 + e]; }
    }
#pragma unroll
    for (int u = 0; u < HP_STG; ++u) {
      const int pos = u * 64 + wid * 8 + (lane & 7);
      if (pos >= NPOS) continue;
      uint4 o = stg[u];
      if constexpr (AFF != 0) {
        float f[8];
        unpack8(o, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = __builtin_fmaf(f[e], sc[e], sh[e]);
        o = pack8_fast(f);
        if constexpr (AFF == 2) o = relu_e16x8(o);
        const int h = r0 - 1 + ((hcode[u] >> 16) & 255);
        if (!((hcode[u] >> 24) && (unsigned)h < (unsigned)H)) o = uint4{0, 0, 0, 0};   // padding stays zero
      }
      *reinterpret_cast<uint4*>(HI + (cg * NPOSP + pos) * 16) = o;
    }
  };

  // ---- this wave's position blocks: NBLK = ceil(P/16) split 4 ways as evenly as possible
  const int NBLK = (P + 15) >> 4;
  const int q4 = NBLK >> 2, r4 = NBLK & 3;
  const int b0 = wm < r4 ? wm * (q4 + 1) : r4 * (q4 + 1) + (wm - r4) * q4;
  const int nb = q4 + (wm < r4 ? 1 : 0);   // live blocks (<= 4 for P <= 224)
  int abase[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int pl = min((b0 + i) * 16 + fr, P - 1);
    const int h = pl / W, w = pl - h * W;
    abase[i] = (fg * NPOSP + (h + 1) * PW + (w + 1)) * 16;
  }
  const int wbase = fg * 1024 + (32 * wn + fr) * 16;   // + s * 4096 + j * 256

  // one tile: halo (in `cur`) -> LDS, prefetch tile t + 1 into `nxt` (the loop is unrolled by two so each register
  // set is a compile-time array; prefetching two tiles ahead measured no faster), MFMAs, epilogue
  auto tile = [&](int t, uint4 (&cur)[HP_STG], uint4 (&nxt)[HP_STG]) {
    __syncthreads();   // previous tile's MFMA reads of HI are done (and, first time, the weight / table writes)
    store_halo(t, cur);
    __syncthreads();
    const int frame = t / tpf, r0 = (t - frame * tpf) * R;
    const size_t row0 = (size_t)frame * H * W + (size_t)r0 * W;
    // EPI 1: this tile's y0 rows are requested BEFORE the prefetch, so the epilogue's wait does not cover it
    uint2 y0v[4][2];
    if constexpr (EPI == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pl = min((b0 + i) * 16 + fr, P - 1);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          y0v[i][j] = *reinterpret_cast<const uint2*>(p.ey0 + (row0 + pl) * C + 32 * wn + 16 * j + 4 * fg);
      }
    }
    if (t + 1 < t_end) load_halo(t + 1, nxt);

    // every wave runs 4 position blocks (a 3-block wave's 4th block re-reads clamped positions and is not stored):
    // branch-free k loop, fragments of step s+1 read while the 8 MFMAs of step s run
    f32x4_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    ev8_t wa[2][2], xb[2][4];
    auto frag = [&](int s, int c) {
      const int jh = (s >> 1) / 3, jw = (s >> 1) % 3;   // (s is a compile-time constant of the unrolled loop)
      const int ao = ((-DIR + DIR * jh) * PW + (-DIR + DIR * jw)) * 16 + (s & 1) * 4 * NPOSP * 16;
#pragma unroll
      for (int j = 0; j < 2; ++j) wa[c][j] = *reinterpret_cast<const ev8_t*>(WI + s * 4096 + j * 256 + wbase);
#pragma unroll
      for (int i = 0; i < 4; ++i) xb[c][i] = *reinterpret_cast<const ev8_t*>(HI + abase[i] + ao);
    };
    frag(0, 0);
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      const int c = s & 1;
      if (s + 1 < 18) {
        frag(s + 1, c ^ 1);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = PVA_MFMA16(wa[c][j], xb[c][i], acc[i][j], 0, 0, 0);
    }

    // ---- epilogue: lane holds channels 32 wn + 16 j + 4 fg + r of position (b0 + i) * 16 + fr
    float s1[2][4], s2[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pl = (b0 + i) * 16 + fr;
      if (i >= nb || pl >= P) continue;
      const size_t row = row0 + pl;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = 32 * wn + 16 * j + 4 * fg;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        float a[4];
        if constexpr (EPI == 1) {
          unpack4(y0v[i][j], a);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (a[r] * bnp[2 * C + n + r] + bnp[3 * C + n + r] > 0.f) ? v[r] : 0.f;
        }
        const uint2 pk = pack4(v);
        *reinterpret_cast<uint2*>(p.y + row * p.ldy + n) = pk;
        float q[4];
        unpack4(pk, q);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1[j][r] += q[r];
          if constexpr (EPI == 1) s2[j][r] += q[r] * a[r];
          else s2[j][r] += q[r] * q[r];
        }
      }
    }
    if (EPI == 0 && p.stats == nullptr) return;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = sum16(s1[j][r]), b = sum16(s2[j][r]);
        if (fr == 0) {
          const int n = 32 * wn + 16 * j + 4 * fg + r;
          red[(wm * 3) * C + n] = a;
          red[(wm * 3 + 1) * C + n] = b;
        }
      }
    __syncthreads();
    if (tid < C) {
      const int n = tid;
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m) { a += red[(m * 3) * C + n]; b += red[(m * 3 + 1) * C + n]; }
      if constexpr (EPI == 0) {
        p.stats[((size_t)t * 2) * C + n] = a;
        p.stats[((size_t)t * 2 + 1) * C + n] = b;
      } else {
        p.epart[((size_t)t * 3) * C + n] = a;
        p.epart[((size_t)t * 3 + 1) * C + n] = (b - bnp[n] * a) * bnp[C + n];
        p.epart[((size_t)t * 3 + 2) * C + n] = 0.f;
      }
    }
  };

  uint4 stgA[HP_STG], stgB[HP_STG];
  if (t_begin < t_end) load_halo(t_begin, stgA);
  for (int t = t_begin; t < t_end; t += 2) {
    tile(t, stgA, stgB);
    if (t + 1 < t_end) tile(t + 1, stgB, stgA);
  }
}

template <int EPI, int AFF, int DIR, int WW, int RR>
void launch_halo64p_t(const ConvParams& p, int cfg, hipStream_t st) {
  const int ntiles = p.M / (RR * WW);
  const size_t lds = 18 * 4 * 64 * 16 + (size_t)8 * hp_nposp(RR, WW) * 16 + (4 * 3 + 4 + 2) * 64 * 4;
  const int cap = (cfg & 4) ? 1024 : 256;   // one workgroup per CU (LDS-bound); 4x that for load balance
  const int grid = ntiles < cap ? ntiles : cap;
  hipLaunchKernelGGL((conv_halo64p_kernel<EPI, AFF, DIR, WW, RR>), dim3(grid), dim3(HP_THREADS), lds, st, p, ntiles);
}

template <int EPI, int AFF, int DIR>
void launch_halo64p(const ConvParams& p, int cfg, hipStream_t st) {
  if (p.Rw == 56) launch_halo64p_t<EPI, AFF, DIR, 56, 4>(p, cfg, st);
  else launch_halo64p_t<EPI, AFF, DIR, 64, 2>(p, cfg, st);
}


// ------------------------------------------------------------------------------------------------------------------
// Double-buffered 64 -> 64 channel variant (launch-word bits 1 + 3; slow res2 conv_b at 56x56).  The persistent
// kernel above runs each tile as three serialised phases — halo store (VALU + ds_write, no MFMA), 18 k-steps of MFMA
// at 0.75 LDS reads per MFMA with two waves per SIMD, epilogue — at 28-31 % MFMA busy (profiles/r6_pmc).  Here:
//   * tiles are 8 rows x 28 columns (P = 224 as before; the halo is 10 x 30 = 300 positions, 1.34x the outputs
//     instead of 1.55x), so TWO halo images fit next to the 72 KB of LDS-resident weights: tile t+1's halo is written
//     (BN+ReLU applied) one chunk per k-step behind tile t's MFMAs, and each tile has one barrier;
//   * 8 waves (two per SIMD, so one wave's staging and epilogue overlap the other's MFMAs) = 4 position groups x 2
//     channel halves, each 4 position blocks x 32 channels, the fragments of step s+1 read during step s;
//   * a staging register is refilled with tile t+2's chunk as soon as it is written, so every global load has a
//     whole tile of latency to hide.
// Epilogues as conv_halo64p_kernel (EPI 0 raw output + BN partial sums per tile, EPI 1 dgrad with the BN_a ReLU mask
// from y0 and the BN_a backward partials).
constexpr int HD_THREADS = 512, HD_R = 8, HD_CW = 28;
constexpr int HD_PW = HD_CW + 2, HD_NPOS = (HD_R + 2) * HD_PW, HD_NPOSP = (HD_NPOS + 15) & ~15;
constexpr int HD_STG = (HD_NPOSP * 8 + HD_THREADS - 1) / HD_THREADS;   // 16-B halo chunks per thread (10)
constexpr int HD_HALO = 8 * HD_NPOSP * 16;                             // bytes of one halo image
constexpr int HD_WI = 18 * 4 * 64 * 16;                                // weight image
constexpr size_t HD_LDS = HD_WI + 2 * HD_HALO + (2 * 4 * 2 + 4) * 64 * 4;
static_assert(HD_LDS <= 160 * 1024, "double-buffered halo tile exceeds LDS");

template <int EPI, int AFF, int DIR>
__global__ __launch_bounds__(HD_THREADS, 1) void conv_halo64d_kernel(const ConvParams p, const int ntiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int C = 64, W = 56;
  char* WI = smem;                                                // [18][4][64][16 B] weights
  char* HI = smem + HD_WI;                                        // [2][8][NPOSP][16 B] halo images
  float* red = reinterpret_cast<float*>(HI + 2 * HD_HALO);        // [2][4 position groups][2][64]
  float* bnp = red + 2 * 4 * 2 * C;                               // EPI 1: [4][64] mean0 rstd0 msc msh
  const int H = p.Rh;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int wn = wid & 1, wm = wid >> 1;
  const int t_begin = (int)((long long)blockIdx.x * ntiles / gridDim.x);
  const int t_end = (int)((long long)(blockIdx.x + 1) * ntiles / gridDim.x);
  const int tpf = (H / HD_R) * 2;   // tiles per frame: row bands x two column halves

  // ---- weights -> LDS (as conv_halo64p_kernel): chunk q = (k-step s, channel group g, output channel n)
  int wtap[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int jh = tap / 3, jw = tap - jh * 3;
    wtap[tap] = (p.bt0 * p.kh + p.bh0 + jh * p.bhs) * p.kw + p.bw0 + jw * p.bws;
  }
  for (int q = tid; q < 18 * 4 * 64; q += HD_THREADS) {
    const int s = q >> 8, g = (q >> 6) & 3, n = q & 63;
    const int tap = s >> 1, half = s & 1;
    int wt = 0;
#pragma unroll
    for (int u = 0; u < 9; ++u) wt = (u == tap) ? wtap[u] : wt;
    *reinterpret_cast<uint4*>(WI + q * 16) =
        *reinterpret_cast<const uint4*>(p.w + (size_t)n * p.Kfull + wt * C + half * 32 + g * 8);
  }
  if constexpr (EPI == 1) {
    for (int i = tid; i < C; i += HD_THREADS) {
      bnp[i] = p.emean0[i]; bnp[C + i] = p.erstd0[i]; bnp[2 * C + i] = p.emsc[i]; bnp[3 * C + i] = p.emsh[i];
    }
  }
  // ---- staging roles: channel group cg = lane >> 3, halo position u*64 + wid*8 + (lane & 7) of chunk u
  const int cg = lane >> 3;
  float sc[8], sh[8];
  if constexpr (AFF != 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { sc[e] = p.in_scale[cg * 8 + e]; sh[e] = p.in_shift[cg * 8 + e]; }
  }
  // halo row (bits 8-15) and column (bits 0-7) of each chunk, bit 16: a real halo position
  int hcode[HD_STG];
#pragma unroll
  for (int u = 0; u < HD_STG; ++u) {
    const int pos = u * 64 + wid * 8 + (lane & 7);
    const int h = pos / HD_PW, w = pos - h * HD_PW;
    hcode[u] = pos < HD_NPOS ? ((1 << 16) | (h << 8) | w) : 0;
  }
  // image row of chunk u in tile t (clamped into the image) and whether it lies inside the image
  auto chunk_at = [&](int t, int u, size_t& row, bool& ok) {
    const int frame = t / tpf, rem = t - frame * tpf;
    const int r = (rem >> 1) * HD_R - 1 + ((hcode[u] >> 8) & 255);
    const int c = (rem & 1) * HD_CW - 1 + (hcode[u] & 255);
    ok = (hcode[u] >> 16) && (unsigned)r < (unsigned)H && (unsigned)c < (unsigned)W;
    row = (size_t)frame * H * W + (size_t)(ok ? r : 0) * W + (ok ? c : 0);
  };
  // staging registers as native vectors and unconditional loads from clamped addresses: no branch around a load, so
  // the wait before each chunk's LDS write counts only the loads issued after it (a predicated load made the
  // compiler wait for every outstanding load — the chunk just requested for tile t+2 included)
  typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
  u32x4_t stg[HD_STG];
  unsigned okm = 0;   // bit u: chunk u of the staged tile lies inside the image
  auto load_chunk = [&](int t, int u) {
    size_t row;
    bool ok;
    chunk_at(t, u, row, ok);
    stg[u] = *reinterpret_cast<const u32x4_t*>(p.x + row * p.ldx + cg * 8);
    okm = ok ? (okm | (1u << u)) : (okm & ~(1u << u));
  };
  auto store_chunk = [&](int u, char* img) {
    if (!(hcode[u] >> 16)) return;
    const bool ok = (okm >> u) & 1u;
    uint4 o = __builtin_bit_cast(uint4, stg[u]);
    if constexpr (AFF != 0) {
      float f[8];
      unpack8(o, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = __builtin_fmaf(f[e], sc[e], sh[e]);
      o = pack8_fast(f);
      if constexpr (AFF == 2) o = relu_e16x8(o);
    }
    const u32x4_t z = {0u, 0u, 0u, 0u};
    const u32x4_t ov = ok ? __builtin_bit_cast(u32x4_t, o) : z;   // padding stays zero
    const int pos = u * 64 + wid * 8 + (lane & 7);
    *reinterpret_cast<u32x4_t*>(img + (cg * HD_NPOSP + pos) * 16) = ov;
  };

  // ---- this wave's position blocks: 14 blocks of 16 as 4 + 4 + 3 + 3 (a 3-block wave's 4th block re-reads block
  // 13 and is not stored).  A fragment's 16 positions must sit on 16 distinct 16-B LDS units, unit(h, w) =
  // (h * 30 + w + 31) mod 16: blocks 0-7 are the first 16 columns of rows 0-7; the 12-column row remnants are paired
  // into blocks 8-13 from rows h, h+2, h+4, h+6 (whose units start 4 lower per two rows), e.g. row h columns 16-27 +
  // row h+2 columns 16-19 — no block straddles a row end the way consecutive positions would
  const int b0 = wm < 2 ? wm * 4 : 8 + (wm - 2) * 3;
  const int nb = wm < 2 ? 4 : 3;
  int abase[4], ph[4], pw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = min(b0 + i, 13);
    int h, w;
    if (b < 8) {
      h = b;
      w = fr;
    } else {
      const int k = b - 8, hb = k / 3, sub = k - hb * 3;
      const int cut = 12 - 4 * sub;   // lanes [0, cut) from row hb + 2 sub, columns 16 + 4 sub ...
      h = hb + 2 * sub + (fr < cut ? 0 : 2);
      w = fr < cut ? 16 + 4 * sub + fr : 16 + fr - cut;
    }
    ph[i] = h;
    pw[i] = w;
    abase[i] = (fg * HD_NPOSP + (h + 1) * HD_PW + (w + 1)) * 16;
  }
  const int wbase = fg * 1024 + (32 * wn + fr) * 16;   // + s * 4096 + j * 256

  // prologue: first tile's halo into image 0, the second tile's chunks into the staging registers
  if (t_begin < t_end) {
#pragma unroll
    for (int u = 0; u < HD_STG; ++u) load_chunk(t_begin, u);
#pragma unroll
    for (int u = 0; u < HD_STG; ++u) store_chunk(u, HI);
#pragma unroll
    for (int u = 0; u < HD_STG; ++u) load_chunk(t_begin + 1 < t_end ? t_begin + 1 : t_begin, u);
  }
  __syncthreads();

  for (int t = t_begin; t < t_end; ++t) {
    const int cur = (t - t_begin) & 1;
    const char* img = HI + cur * HD_HALO;
    char* nxt = HI + (cur ^ 1) * HD_HALO;
    const bool has1 = t + 1 < t_end, has2 = t + 2 < t_end;
    const int frame = t / tpf, rem = t - frame * tpf;
    const int r0 = (rem >> 1) * HD_R, c0 = (rem & 1) * HD_CW;
    const size_t fbase = (size_t)frame * H * W;
    uint2 y0v[4][2];
    if constexpr (EPI == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const size_t row = fbase + (size_t)(r0 + ph[i]) * W + c0 + pw[i];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          y0v[i][j] = *reinterpret_cast<const uint2*>(p.ey0 + row * C + 32 * wn + 16 * j + 4 * fg);
      }
    }
    f32x4_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    ev8_t wa[2][2], xb[2][4];
    auto frag = [&](int s, int c) {
      const int jh = (s >> 1) / 3, jw = (s >> 1) % 3;
      const int ao = ((-DIR + DIR * jh) * HD_PW + (-DIR + DIR * jw)) * 16 + (s & 1) * 4 * HD_NPOSP * 16;
#pragma unroll
      for (int j = 0; j < 2; ++j) wa[c][j] = *reinterpret_cast<const ev8_t*>(WI + s * 4096 + j * 256 + wbase);
#pragma unroll
      for (int i = 0; i < 4; ++i) xb[c][i] = *reinterpret_cast<const ev8_t*>(img + abase[i] + ao);
    };
    frag(0, 0);
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      const int c = s & 1;
      if (s + 1 < 18) {
        frag(s + 1, c ^ 1);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = PVA_MFMA16(wa[c][j], xb[c][i], acc[i][j], 0, 0, 0);
      // next tile's halo chunk s-2 -> the other image, then its register takes tile t+2's chunk
      if (s >= 2 && s - 2 < HD_STG) {
        __builtin_amdgcn_sched_barrier(0);
        if (has1) store_chunk(s - 2, nxt);
        load_chunk(has2 ? t + 2 : t, s - 2);   // (past the range: a harmless reload of this tile)
      }
    }

    // ---- epilogue: lane holds channels 32 wn + 16 j + 4 fg + r of position (b0 + i) * 16 + fr
    float s1[2][4], s2[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i >= nb) continue;
      const size_t row = fbase + (size_t)(r0 + ph[i]) * W + c0 + pw[i];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = 32 * wn + 16 * j + 4 * fg;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        float a[4];
        if constexpr (EPI == 1) {
          unpack4(y0v[i][j], a);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (a[r] * bnp[2 * C + n + r] + bnp[3 * C + n + r] > 0.f) ? v[r] : 0.f;
        }
        const uint2 pk = pack4(v);
        *reinterpret_cast<uint2*>(p.y + row * p.ldy + n) = pk;
        float q[4];
        unpack4(pk, q);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1[j][r] += q[r];
          if constexpr (EPI == 1) s2[j][r] += q[r] * a[r];
          else s2[j][r] += q[r] * q[r];
        }
      }
    }
    float* rb = red + cur * (4 * 2 * C);
    const bool want = !(EPI == 0 && p.stats == nullptr);
    if (want) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float a = sum16(s1[j][r]), b = sum16(s2[j][r]);
          if (fr == 0) {
            const int n = 32 * wn + 16 * j + 4 * fg + r;
            rb[(wm * 2) * C + n] = a;
            rb[(wm * 2 + 1) * C + n] = b;
          }
        }
    }
    __syncthreads();   // next image written, this image read by every wave, partials complete
    if (want && tid < C) {
      const int n = tid;
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m) { a += rb[(m * 2) * C + n]; b += rb[(m * 2 + 1) * C + n]; }
      if constexpr (EPI == 0) {
        p.stats[((size_t)t * 2) * C + n] = a;
        p.stats[((size_t)t * 2 + 1) * C + n] = b;
      } else {
        p.epart[((size_t)t * 3) * C + n] = a;
        p.epart[((size_t)t * 3 + 1) * C + n] = (b - bnp[n] * a) * bnp[C + n];
        p.epart[((size_t)t * 3 + 2) * C + n] = 0.f;
      }
    }
  }
}

template <int EPI, int AFF, int DIR>
void launch_halo64d(const ConvParams& p, int cfg, hipStream_t st) {
  const int ntiles = p.M / (HD_R * HD_CW);
  const int cap = (cfg & 4) ? 1024 : 256;   // one workgroup per CU (LDS-bound); 4x that for load balance
  const int grid = ntiles < cap ? ntiles : cap;
  hipLaunchKernelGGL((conv_halo64d_kernel<EPI, AFF, DIR>), dim3(grid), dim3(HD_THREADS), HD_LDS, st, p, ntiles);
}


// ------------------------------------------------------------------------------------------------------------------
// Narrow variant (fast pathway: 8 / 16 / 32 channels in and out, P = R*W <= 1024 positions per tile).  At these
// widths the conv is a pure streaming problem (K = 9*C <= 288): the halo [(R+2) x (W+2)][C] is staged once
// (position-major, 16/32/64 B per position), the weights of every k-step live in registers for the whole kernel,
// and each wave walks 16-position blocks of the tile: a k-step covers 32/C taps, lane group g (= lane >> 4) reads its
// own tap's 16 B of channels at (position + tap offset) straight into the MFMA operand (the 9 taps padded to whole
// k-steps with zero weights), so one LDS read per lane feeds each MFMA and nothing is re-gathered from L2.
constexpr int HN_PMAX = 1024;

__host__ __device__ inline int halo_rows_narrow(int H, int W) {
  for (int r = H; r >= 1; --r)
    if (H % r == 0 && r * W <= HN_PMAX) return r;
  return 0;
}

template <int CG, int NN, int EPI, int AFF>
__global__ __launch_bounds__(HC_THREADS) void conv_halo_narrow_kernel(const ConvParams p, const int R) {
  constexpr int NB = (NN + 15) / 16;          // 16-channel output blocks
  constexpr int GPT = CG / 8;                 // 16-B channel groups per tap
  constexpr int TPS = 4 / GPT;                // taps per 32-wide k-step
  constexpr int NSTEP = (9 + TPS - 1) / TPS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int W = p.Rw, H = p.Rh, PW = W + 2;
  const int P = R * W;
  const int NPOS = (R + 2) * PW;
  char* box = smem;                                                        // [NPOS][CG]
  float* red = reinterpret_cast<float*>(smem + ((NPOS * CG * 2 + 15) & ~15));   // [4 waves][2|3][NN]
  float* aff = red + (EPI ? 3 : 2) * 4 * NN;                               // [2][CG]
  float* bnp = aff + 2 * CG;                                               // EPI 1: [4][NN]

  const int tile_m = xcd_remap(blockIdx.x, gridDim.x);
  const int tpf = H / R;
  const int frame = tile_m / tpf, r0 = (tile_m - frame * tpf) * R;
  const int fbase = frame * H * W;
  if constexpr (AFF != 0) {
    for (int i = tid; i < CG; i += HC_THREADS) { aff[i] = p.in_scale[i]; aff[CG + i] = p.in_shift[i]; }
  }
  if constexpr (EPI == 1) {
    for (int i = tid; i < NN; i += HC_THREADS) {
      bnp[i] = p.emean0[i]; bnp[NN + i] = p.erstd0[i]; bnp[2 * NN + i] = p.emsc[i]; bnp[3 * NN + i] = p.emsh[i];
    }
  }
  // this lane's weights of every k-step (A operand: row = output channel, 8 k = 8 channels of its group's tap)
  ev8_t wf[NSTEP][NB];
  int toff[NSTEP];
  const int chb = (fg % GPT) * 16;
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) {
    const int tap = s * TPS + fg / GPT;
    const bool real = tap < 9;
    const int jh = real ? tap / 3 : 1, jw = real ? tap - (tap / 3) * 3 : 1;
    toff[s] = real ? ((p.aoh + p.dir * jh) * PW + (p.aow + p.dir * jw)) * (CG * 2) : 0;
    const int wt = (p.bt0 * p.kh + p.bh0 + jh * p.bhs) * p.kw + p.bw0 + jw * p.bws;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int co = j * 16 + fr;
      uint4 v = uint4{0, 0, 0, 0};
      if (real && co < p.Ngemm) v = *reinterpret_cast<const uint4*>(p.w + (size_t)co * p.Kfull + wt * CG + (fg % GPT) * 8);
      wf[s][j] = __builtin_bit_cast(ev8_t, v);
    }
  }
  __syncthreads();
  // ---- stage the halo: chunk c -> box position c / GPT, channel group c % GPT (fixed per thread)
  {
    const int cgp = tid % GPT;
    float sc[8], sh[8];
    if constexpr (AFF != 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { sc[e] = aff[cgp * 8 + e]; sh[e] = aff[CG + cgp * 8 + e]; }
    }
    constexpr int PPP = HC_THREADS / GPT;   // box positions per pass
    const int b_first = tid / GPT;
    int hh = b_first / PW, ww = b_first - (b_first / PW) * PW;
    constexpr int BATCH = 4;
    for (int b0 = b_first; b0 < NPOS; b0 += BATCH * PPP) {
      uint4 v[BATCH];
      bool ok[BATCH];
#pragma unroll
      for (int u = 0; u < BATCH; ++u) {
        const int h = r0 - 1 + hh, w = ww - 1;
        ok[u] = b0 + u * PPP < NPOS && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        v[u] = ok[u] ? *reinterpret_cast<const uint4*>(p.x + (size_t)(fbase + h * W + w) * p.ldx + cgp * 8)
                     : uint4{0, 0, 0, 0};
        ww += PPP;
        while (ww >= PW) { ww -= PW; ++hh; }
      }
#pragma unroll
      for (int u = 0; u < BATCH; ++u) {
        const int bb = b0 + u * PPP;
        if (bb >= NPOS) break;
        uint4 o = v[u];
        if constexpr (AFF != 0) {
          float f[8];
          unpack8(o, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = __builtin_fmaf(f[e], sc[e], sh[e]);
          o = pack8_fast(f);
          if constexpr (AFF == 2) o = relu_e16x8(o);
          if (!ok[u]) o = uint4{0, 0, 0, 0};
        }
        *reinterpret_cast<uint4*>(box + bb * (CG * 2) + cgp * 16) = o;
      }
    }
  }
  __syncthreads();
  // ---- 16-position blocks, round-robin over the waves
  float s1[NB][4], s2[NB][4];
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
  const int MB = (P + 15) / 16;
  for (int mb = wid; mb < MB; mb += 4) {
    const int pl = mb * 16 + fr;
    const int pc = min(pl, P - 1);
    const int h = pc / W, w = pc - h * W;
    const char* src = box + ((h + 1) * PW + (w + 1)) * (CG * 2) + chb;
    f32x4_t acc[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      const ev8_t xf = *reinterpret_cast<const ev8_t*>(src + toff[s]);
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[j] = PVA_MFMA16(wf[s][j], xf, acc[j], 0, 0, 0);
    }
    if (pl >= P) continue;
    const int row = fbase + r0 * W + pl;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int n = j * 16 + 4 * fg;
      if (n >= NN) continue;
      float v[4] = {acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
      float a[4];
      if constexpr (EPI == 1) {
        unpack4(*reinterpret_cast<const uint2*>(p.ey0 + (size_t)row * NN + n), a);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (a[r] * bnp[2 * NN + n + r] + bnp[3 * NN + n + r] > 0.f) ? v[r] : 0.f;
      }
      const uint2 pk = pack4(v);
      *reinterpret_cast<uint2*>(p.y + (size_t)row * p.ldy + n) = pk;
      float q[4];
      unpack4(pk, q);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s1[j][r] += q[r];
        if constexpr (EPI == 1) s2[j][r] += q[r] * a[r]; else s2[j][r] += q[r] * q[r];
      }
    }
  }
  // ---- per-tile partial sums (EPI 0: sum, sum of squares; EPI 1: sum v, sum v*xhat0, 0)
  if (EPI == 0 && p.stats == nullptr) return;
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a = sum16(s1[j][r]), b = sum16(s2[j][r]);
      const int n = j * 16 + 4 * fg + r;
      if (fr == 0 && n < NN) {
        red[(wid * 2) * NN + n] = a;
        red[(wid * 2 + 1) * NN + n] = b;
      }
    }
  __syncthreads();
  for (int n = tid; n < NN; n += HC_THREADS) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) { a += red[(w * 2) * NN + n]; b += red[(w * 2 + 1) * NN + n]; }
    if constexpr (EPI == 0) {
      p.stats[(tile_m * 2) * NN + n] = a;
      p.stats[(tile_m * 2 + 1) * NN + n] = b;
    } else {
      p.epart[(tile_m * 3) * NN + n] = a;
      p.epart[(tile_m * 3 + 1) * NN + n] = (b - bnp[n] * a) * bnp[NN + n];
      p.epart[(tile_m * 3 + 2) * NN + n] = 0.f;
    }
  }
}

template <int CG, int NN>
void launch_narrow(const ConvParams& p, hipStream_t st) {
  const int R = halo_rows_narrow(p.Rh, p.Rw);
  const int NPOS = (R + 2) * (p.Rw + 2);
  const bool epi = p.epart != nullptr;
  const size_t lds = ((size_t)NPOS * CG * 2 + 15) / 16 * 16 + (size_t)(epi ? 3 : 2) * 4 * NN * 4 + 2 * CG * 4 +
                     4 * NN * 4;
  const dim3 grid(p.M / (R * p.Rw)), block(HC_THREADS);
  if (epi) { hipLaunchKernelGGL((conv_halo_narrow_kernel<CG, NN, 1, 0>), grid, block, lds, st, p, R); return; }
  switch (p.affine) {
    case 0: hipLaunchKernelGGL((conv_halo_narrow_kernel<CG, NN, 0, 0>), grid, block, lds, st, p, R); break;
    case 1: hipLaunchKernelGGL((conv_halo_narrow_kernel<CG, NN, 0, 1>), grid, block, lds, st, p, R); break;
    default: hipLaunchKernelGGL((conv_halo_narrow_kernel<CG, NN, 0, 2>), grid, block, lds, st, p, R); break;
  }
}

}  // namespace

// Positions per tile when the halo kernel can run this launch's geometry, else 0.  Geometry only: the epilogue
// conditions (no accumulate / residual / bias / ReLU bits) are checked by conv_halo_epi_ok.
int conv_halo_legal(const ConvParams& p, int chunk) {
  if (chunk != 8 || p.nt != 1 || p.nh != 3 || p.nw != 3) return 0;
  if (p.Rt != p.Gt || p.Rt != p.Ot || p.Rh != p.Gh || p.Rh != p.Oh || p.Rw != p.Gw || p.Rw != p.Ow) return 0;
  if (p.ost != 1 || p.osh != 1 || p.osw != 1 || p.ort || p.orh || p.orw) return 0;
  if (p.ast != 1 || p.ash != 1 || p.asw != 1 || p.aot != 0) return 0;
  // every tap offset within the one-position halo
  for (int j = 0; j < 3; ++j) {
    const int dh = p.aoh + p.dir * j, dw = p.aow + p.dir * j;
    if (dh < -1 || dh > 1 || dw < -1 || dw > 1) return 0;
  }
  if (p.ldx % 8 != 0 || p.ldy % 4 != 0 || p.M % (p.Rh * p.Rw) != 0) return 0;
  const bool narrow = (p.Cg == 8 || p.Cg == 16 || p.Cg == 32) && (p.Ngemm == 8 || p.Ngemm == 16 || p.Ngemm == 32);
  if (narrow) {   // conv_halo_narrow_kernel (fast pathway)
    const int R = halo_rows_narrow(p.Rh, p.Rw);
    return (R > 0 && R * p.Rw >= 128) ? R * p.Rw : 0;
  }
  if (p.Cg % 32 != 0 || (p.Cg > 128 && p.Cg % 128 != 0) || p.Ngemm % 64 != 0) return 0;
  const int R = halo_rows(p.Rh, p.Rw);
  // at least 128 positions per tile: the callers size the BN partial-sum slabs for 128-row tiles
  if (R == 0 || R * p.Rw < 128 || p.M % (p.Rh * p.Rw) != 0) return 0;
  return R * p.Rw;
}

// 1 when the persistent 64-channel variant (launch-word bit 1) can run this geometry (conv_halo_legal > 0 too), 2 when
// the double-buffered variant (bits 1 + 3: 56-wide images, 8-row bands, the same 224-position tiles) can as well
int conv_halo64p_legal(const ConvParams& p, int chunk) {
  if (p.Cg != 64 || p.Ngemm != 64 || p.Kfull < 9 * 64 || conv_halo_legal(p, chunk) <= 0) return 0;
  if (!((p.dir == 1 && p.aoh == -1 && p.aow == -1) || (p.dir == -1 && p.aoh == 1 && p.aow == 1))) return 0;
  const int R = halo_rows(p.Rh, p.Rw);   // instantiated image widths: 56 (224 crop) and 64 (R101's 256 crop)
  if (p.epart && p.dir != -1) return 0;
  if (p.Rw == 56 && R == 4) return p.Rh % HD_R == 0 ? 2 : 1;
  return (p.Rw == 64 && R == 2) ? 1 : 0;
}

int conv_halo_epi_ok(const ConvParams& p) {
  if (p.accum || p.fres || p.ebias || p.nostore || p.eres || p.emask || p.ey1) return 0;
  const bool epi = p.epart != nullptr;
  if (epi) return (p.ey0 && p.emsc && p.emsh && p.emean0 && p.erstd0 && !p.affine) ? 1 : 0;
  return 1;
}

void conv_halo_launch(const ConvParams& p, int cfg, hipStream_t st) {
  if (p.Cg <= 32 && p.Ngemm <= 32) {
    const int key = p.Cg * 100 + p.Ngemm;
    switch (key) {
      case 808: launch_narrow<8, 8>(p, st); break;
      case 816: launch_narrow<8, 16>(p, st); break;
      case 832: launch_narrow<8, 32>(p, st); break;
      case 1608: launch_narrow<16, 8>(p, st); break;
      case 1616: launch_narrow<16, 16>(p, st); break;
      case 1632: launch_narrow<16, 32>(p, st); break;
      case 3208: launch_narrow<32, 8>(p, st); break;
      case 3216: launch_narrow<32, 16>(p, st); break;
      default: launch_narrow<32, 32>(p, st); break;
    }
    return;
  }
  const int R = halo_rows(p.Rh, p.Rw);
  const bool epi = p.epart != nullptr;
  if ((cfg & 2) && (cfg & 8)) {   // double-buffered 64-channel variant (legality: conv_halo64p_legal == 2)
    if (epi) launch_halo64d<1, 0, -1>(p, cfg, st);
    else if (p.dir < 0) launch_halo64d<0, 0, -1>(p, cfg, st);
    else if (p.affine == 0) launch_halo64d<0, 0, 1>(p, cfg, st);
    else if (p.affine == 1) launch_halo64d<0, 1, 1>(p, cfg, st);
    else launch_halo64d<0, 2, 1>(p, cfg, st);
    return;
  }
  if (cfg & 2) {   // persistent 64-channel variant (legality checked by the bindings: conv_halo64p_legal)
    if (epi) launch_halo64p<1, 0, -1>(p, cfg, st);
    else if (p.dir < 0) launch_halo64p<0, 0, -1>(p, cfg, st);
    else if (p.affine == 0) launch_halo64p<0, 0, 1>(p, cfg, st);
    else if (p.affine == 1) launch_halo64p<0, 1, 1>(p, cfg, st);
    else launch_halo64p<0, 2, 1>(p, cfg, st);
    return;
  }
  if ((cfg & 1) || p.Ngemm % 128 != 0) launch_ntile<64>(p, R, epi, st);
  else launch_ntile<128>(p, R, epi, st);
}

PVA_NS_END  // namespace PVA_NS
