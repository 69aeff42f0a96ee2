// Implicit-GEMM 3-D convolution on MFMA (gfx950): forward and dgrad.
//
// Layout: activations NDHWC bf16 (channels contiguous, arbitrary row stride so channel slices of a
// concatenated tensor are zero-copy views); weights packed K-contiguous [Ngemm][taps][C].
// One kernel template serves every conv class of SlowFast/Slow:
//   * k is ordered (tap, channel), so each 16-B (8 x bf16) or 8-B (4 x bf16, stems with RGB0 input)
//     chunk of a tile row is one contiguous global load of one tap; padding taps load zeros.
//   * A (gathered activations) and B (weights) are register-staged into a double-buffered LDS tile
//     (BK = 32 or 64) through a one-stage-ahead register ring (tile s+1 is written to LDS right after the
//     barrier of step s, tile s+2 is issued at once: one barrier per k-step, every load gets a whole
//     k-step of MFMA work to land; cdna_hip_programming.md T14), with an XOR slot swizzle that makes every ds_read_b128 fragment read
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

PVA_NS_BEGIN

namespace {

// LDS tile rows are BK bf16 (64 or 128 bytes) of 16-byte slots, XOR-swizzled so that the 16-lane
// groups of every ds_read_b128 fragment read hit 16 distinct slots of the 256-byte bank row
// (brute-force checked against the gfx950 b128 lane groups for both row lengths).
// LDS bytes before the stats/affine area: the double-buffered k tiles, or (EPI) the fp32 output tile.
// NS = k-tile buffers: 2 (register staging) or 3 (LDS-DMA ring, one tile in flight across each barrier)
// EPI 1 stages the fp32 output tile through LDS in slices of epi_rows rows (64 for the 256x256 tile, whose
// whole fp32 tile would not fit)
__host__ __device__ constexpr int epi_rows(int BM, int BN) { return BM * BN > 128 * 128 ? 64 : BM; }

__host__ __device__ constexpr int main_lds_bytes(int BM, int BN, int BK, int EPI, int NS = 2) {
  return (EPI && epi_rows(BM, BN) * (BN * 4 + 16) > NS * (BM + BN) * BK * 2) ? epi_rows(BM, BN) * (BN * 4 + 16)
                                                                             : NS * (BM + BN) * BK * 2;
}

__host__ __device__ constexpr int dma_stages(int BM, int BN, int BK, bool dma) {
  // the 256x256 tile runs one workgroup per CU anyway: at BK = 32 a 4-buffer ring (128 KB, two tiles in flight
  // across each barrier) fits beside its epilogue/statistics area.  The 4-wave 256x128 tile keeps two
  // workgroups per CU (<= 80 KB each: a 3-buffer ring at BK = 32)
  return (dma && BM * BN == 256 * 128) ? (3 * (BM + BN) * BK * 2 <= 80 * 1024 ? 3 : 2)
         : (dma && BM * BN > 128 * 128 && 4 * (BM + BN) * BK * 2 <= 128 * 1024) ? 4
         : (dma && 3 * (BM + BN) * BK * 2 <= 96 * 1024) ? 3 : 2;
}

template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// s_waitcnt vmcnt(BASE + nb) for a wave-uniform runtime nb in [0, MAXB] (the immediate must be a constant)
template <int BASE, int MAXB>
__device__ __forceinline__ void vm_wait_dyn(int nb) {
  if constexpr (MAXB <= 0) {
    vm_wait<BASE>();
  } else {
    if (nb >= MAXB) vm_wait<BASE + MAXB>();
    else vm_wait_dyn<BASE, MAXB - 1>(nb);
  }
}

// 16-B LDS-DMA of one lane: buffer_load_dwordx4 ... lds into wave-uniform LDS address `lds` + 16 * lane
// (the address_space(3) cast only exists in the device pass; the host pass only needs the kernel stub)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
#endif
}

// the XOR applied to a row's 16-B slot index by lds_off (an involution: slot ^ swz ^ swz == slot)
template <int BK>
__device__ __forceinline__ int lds_swz(int row) {
  if constexpr (BK == 32) return ((row >> 2) & 1) << 1;
  else return row & 6;
}

template <int BK>
__device__ __forceinline__ int lds_off(int row, int slot) {
  if constexpr (BK == 32) return row * 64 + ((slot ^ (((row >> 2) & 1) << 1)) << 4);
  else return row * 128 + ((slot ^ (row & 6)) << 4);
}

// MFMAs of one LDS k tile.  The fragments of k-step kk+1 are read while the MFMAs of kk run (register double
// buffer); the scheduling barrier keeps the compiler from sinking those reads back next to their use, where
// each read exposes the LDS latency to the MFMA pipe (the compiler otherwise reads 2 fragments 4 MFMAs ahead).
template <int BK, int TM, int TN>
__device__ __forceinline__ void mma_ktile(const char* A, const int (&fa)[BK / 32][TM], const int (&fb)[BK / 32][TN],
                                          f32x4_t (&acc)[TM][TN]) {
  ev8_t af[2][TM], bfr[2][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) af[0][i] = *reinterpret_cast<const ev8_t*>(A + fa[0][i]);
#pragma unroll
  for (int j = 0; j < TN; ++j) bfr[0][j] = *reinterpret_cast<const ev8_t*>(A + fb[0][j]);
#pragma unroll
  for (int kk = 0; kk < BK / 32; ++kk) {
    const int c = kk & 1;
    if (kk + 1 < BK / 32) {
#pragma unroll
      for (int i = 0; i < TM; ++i) af[c ^ 1][i] = *reinterpret_cast<const ev8_t*>(A + fa[kk + 1][i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[c ^ 1][j] = *reinterpret_cast<const ev8_t*>(A + fb[kk + 1][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = PVA_MFMA16(bfr[c][j], af[c][i], acc[i][j], 0, 0, 0);
  }
}

template <int BM, int BN, int WM, int WN, int CH, int BK, int EPI, int UT>
// the 4-wave 256x128 tile runs two workgroups per CU: at most 256 VGPRs (two waves per SIMD)
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64, (BM * BN == 256 * 128) ? 2 : 1)
void conv_igemm_kernel(const ConvParams p) {
  constexpr int NWN = BN / WN;
  constexpr int NT = (BM / WM) * NWN * 64;
  constexpr int CPR = BK / CH;  // chunks per tile row
  constexpr int A_CHUNKS = BM * CPR, B_CHUNKS = BN * CPR;
  constexpr int A_SLOTS = (A_CHUNKS + NT - 1) / NT;
  constexpr int B_SLOTS = (B_CHUNKS + NT - 1) / NT;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int TILE_BYTES = (BM + BN) * BK * 2;
  constexpr int STG_PITCH = BN * 4 + 16;  // EPI staging row pitch (fp32 tile, padded)
  // LDS-DMA loader: 3-buffer ring when it fits 96 KB (>= 1 more workgroup per CU), else 2 buffers
  constexpr int NSTAGE = dma_stages(BM, BN, BK, (UT & 17) == 17);
  constexpr int MAIN_BYTES = main_lds_bytes(BM, BN, BK, EPI, NSTAGE);
  static_assert(NT % CPR == 0, "thread count must be a multiple of chunks per row");
  using VT = typename std::conditional<CH == 8, uint4, uint2>::type;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  // stats slots, one per wave row (EPI 0: [BM/WM][2][BN]) or per wave (EPI 1: [NW][3][BN]); summed in a fixed
  // order, so the BN statistics are bitwise deterministic (no float atomics)
  constexpr int NWAVES = (BM / WM) * NWN;
  constexpr int RED_FLOATS = EPI >= 1 ? NWAVES * 3 * BN : (BM / WM) * 2 * BN;
  float* red = reinterpret_cast<float*>(smem + MAIN_BYTES);
  float* bnp = red + RED_FLOATS;  // EPI: [6][BN] mean0 rstd0 mean1 rstd1 mask-scale mask-shift
  float* aff = bnp + (EPI >= 1 ? 6 * BN : 0);                            // [2][Cg] affine

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / NWN, wn = wid % NWN;
  const int n_tiles = (p.Ngemm + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int tile_m = t / n_tiles, tile_n = t % n_tiles;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  const bool do_stats = EPI == 0 && p.stats != nullptr;
  const bool do_bstats = EPI >= 1 && p.epart != nullptr;
  const int affine = p.affine;
  if (do_bstats) {  // this tile's BN constants, read once here so the epilogue never waits on them
    for (int i = tid; i < BN; i += NT) {
      const int n = n0 + i;
      const bool ok = n < p.Ngemm, d = ok && p.ey1 != nullptr, d0 = ok && p.ey0 != nullptr;
      bnp[i] = d0 ? p.emean0[n] : 0.f;
      bnp[BN + i] = d0 ? p.erstd0[n] : 0.f;
      bnp[2 * BN + i] = d ? p.emean1[n] : 0.f;
      bnp[3 * BN + i] = d ? p.erstd1[n] : 0.f;
      bnp[4 * BN + i] = (ok && p.emsc) ? p.emsc[n] : 0.f;
      bnp[5 * BN + i] = (ok && p.emsh) ? p.emsh[n] : 0.f;
    }
  }
  if (affine) {
    for (int i = tid; i < p.Cg; i += NT) { aff[i] = p.in_scale[i]; aff[p.Cg + i] = p.in_shift[i]; }
  }

  const int RHW = p.Rh * p.Rw, RTHW = p.Rt * RHW;
  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int frow = lane & 15, fslot = lane >> 4;
  int fa[BK / 32][TM], fb[BK / 32][TN];
#pragma unroll
  for (int kk = 0; kk < BK / 32; ++kk) {
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[kk][i] = lds_off<BK>(wm * WM + i * 16 + frow, fslot + 4 * kk);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[kk][j] = BM * BK * 2 + lds_off<BK>(wn * WN + j * 16 + frow, fslot + 4 * kk);
  }

  if constexpr (UT & 1) {
    // UT bit 1: padding reachable (bounds tests), bits 2-3: consumer-side affine mode — compile-time, so
    // the k-loop is branch-free
    // ================= uniform-tap loader (Cg % BK == 0, CH == 8) =================
    // Every k-step of the block lies inside one tap, so the tap / channel cursor is wave-uniform (SGPRs).
    // Raw buffer loads: weights = per-slot VGPR row offset + SGPR (tap, channel) offset -> no VALU;
    // activations without reachable padding likewise; with padding, a per-slot valid-tap bitmask (built
    // once) picks the row offset or an out-of-range offset (the buffer unit returns zeros).
    static_assert(CH == 8, "uniform-tap loader stages 16-B chunks");
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)p.wbytes, 0x00020000);
    constexpr unsigned OOB = 0xFFFFFFF0u;
    const int col = tid % CPR;
    constexpr bool check = (UT >> 1) & 1;
    constexpr int uaff = (UT >> 2) & 3;
    constexpr bool glds_ut = (UT >> 4) & 1;
    static_assert(!glds_ut || uaff == 0, "LDS-DMA staging cannot transform the A operand");
    const int GHW = p.Gh * p.Gw, GTHW = p.Gt * GHW;
    // most negative tap offset (dgrad walks taps backwards): the no-check form adds taps as a >= 0 soffset
    const int tmin = p.dir < 0 ? -(((p.nt - 1) * p.Gh + (p.nh - 1)) * p.Gw + (p.nw - 1)) * p.ldx : 0;
    int a_vo[A_SLOTS], sa[A_SLOTS];
    unsigned tmask[A_SLOTS];
#pragma unroll
    for (int s = 0; s < A_SLOTS; ++s) {
      const int idx = tid + s * NT;
      const int row = idx / CPR;
      const int m = m0 + row;
      const bool rv = idx < A_CHUNKS && m < p.M;
      int at = 0, ah = 0, aw = 0, off = 0;
      if (rv) {
        const int b = pva_fdiv(m, p.mg_thw, p.sh_thw);
        int r = m - b * RTHW;
        const int qt = pva_fdiv(r, p.mg_hw, p.sh_hw); r -= qt * RHW;
        const int qh = pva_fdiv(r, p.mg_w, p.sh_w); const int qw = r - qh * p.Rw;
        at = qt * p.ast + p.aot; ah = qh * p.ash + p.aoh; aw = qw * p.asw + p.aow;
        // LDS-DMA staging: the lane's LDS slot is `col`, so it loads the logical chunk that the XOR swizzle
        // places there (lds_off: physical slot = logical ^ swz(row), an involution)
        off = (b * GTHW + (at * p.Gh + ah) * p.Gw + aw) * p.ldx + (glds_ut ? col ^ lds_swz<BK>(row) : col) * 8;
      }
      unsigned msk = 0;
      if (check && rv) {
        int t = 0;
        for (int jt = 0; jt < p.nt; ++jt)
          for (int jh = 0; jh < p.nh; ++jh)
            for (int jw = 0; jw < p.nw; ++jw, ++t)
              if ((unsigned)(at + p.dir * jt) < (unsigned)p.Gt && (unsigned)(ah + p.dir * jh) < (unsigned)p.Gh &&
                  (unsigned)(aw + p.dir * jw) < (unsigned)p.Gw)
                msk |= 1u << t;
      }
      tmask[s] = msk;
      // no-check: rows past M read a real (ignored) address — never rely on range checks there
      a_vo[s] = check ? off * 2 : (rv ? (off + tmin) * 2 : 0);
      sa[s] = lds_off<BK>(row, col);
    }
    int b_vo[B_SLOTS], sb[B_SLOTS];
#pragma unroll
    for (int s = 0; s < B_SLOTS; ++s) {
      const int idx = tid + s * NT;
      const int row = idx / CPR;
      const int n = n0 + row;
      const int bcol = glds_ut ? col ^ lds_swz<BK>(row) : col;
      b_vo[s] = (idx < B_CHUNKS && n < p.Ngemm) ? (n * p.Kfull + bcol * 8) * 2 : 0;  // columns >= N: ignored
      sb[s] = lds_off<BK>(row, col);
    }
    // UT bit 5 (LDS-DMA loader only): L2 touch-prefetch of the A rows one k-tile ahead of their LDS-DMA — one 4-byte
    // DMA per 128-B row line into a per-wave dummy LDS slot, so the tile's real DMA finds its lines in L2 (twice the
    // bytes in flight per CU at one instruction per wave and tile).  Always one touch per issued k-tile step (a touch
    // past the last tile re-reads a line or reads out of range: zeros, harmless), so its vmcnt share is constant.
    constexpr bool touch = (UT >> 5) & 1;
    static_assert(!touch || glds_ut, "touch-prefetch rides on the LDS-DMA loader");
    constexpr int TRPW = BM / NWAVES;   // A rows touched per wave
    static_assert(!touch || TRPW <= 64, "one touched row per lane");
    int t_vo = 0;
    unsigned t_msk = 0;
    bool t_on = false;
    if constexpr (touch) {
      const int row = wid * TRPW + lane;
      const int m = m0 + row;
      t_on = lane < TRPW && m < p.M;
      int at = 0, ah = 0, aw = 0, off = 0;
      if (t_on) {
        const int b = pva_fdiv(m, p.mg_thw, p.sh_thw);
        int r = m - b * RTHW;
        const int qt = pva_fdiv(r, p.mg_hw, p.sh_hw); r -= qt * RHW;
        const int qh = pva_fdiv(r, p.mg_w, p.sh_w); const int qw = r - qh * p.Rw;
        at = qt * p.ast + p.aot; ah = qh * p.ash + p.aoh; aw = qw * p.asw + p.aow;
        off = (b * GTHW + (at * p.Gh + ah) * p.Gw + aw) * p.ldx;
        if (check) {
          int t = 0;
          for (int jt = 0; jt < p.nt; ++jt)
            for (int jh = 0; jh < p.nh; ++jh)
              for (int jw = 0; jw < p.nw; ++jw, ++t)
                if ((unsigned)(at + p.dir * jt) < (unsigned)p.Gt && (unsigned)(ah + p.dir * jh) < (unsigned)p.Gh &&
                    (unsigned)(aw + p.dir * jw) < (unsigned)p.Gw)
                  t_msk |= 1u << t;
        }
      }
      t_vo = check ? off * 2 : (off + tmin) * 2;
    }
    // uniform k cursor
    int kt_ = 0, kh_ = 0, kw_ = 0, t_ = 0, kb = 0, tapA = 0, tapW = 0;
    auto retap = [&]() {
      tapA = p.dir * ((kt_ * p.Gh + kh_) * p.Gw + kw_) * p.ldx;
      tapW = (((p.bt0 + kt_ * p.bts) * p.kh + (p.bh0 + kh_ * p.bhs)) * p.kw + (p.bw0 + kw_ * p.bws)) * p.Cg;
    };
    retap();
    uint4 ra[A_SLOTS], rb[B_SLOTS];
    int ra_c = 0;
    unsigned ra_valid = 0;
    auto load = [&]() {
      const int ta = tapA + kb;
      ra_c = kb;
      ra_valid = 0;
#pragma unroll
      for (int s = 0; s < A_SLOTS; ++s) {
        if (check) {
          const bool v = (tmask[s] >> t_) & 1u;
          ra[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, v ? a_vo[s] + ta * 2 : (int)OOB, 0, 0));
          ra_valid |= (unsigned)v << s;
        } else {
          ra[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, a_vo[s], (ta - tmin) * 2, 0));
        }
      }
      const int wso = (tapW + kb) * 2;
#pragma unroll
      for (int s = 0; s < B_SLOTS; ++s)
        rb[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wr, b_vo[s], wso, 0));
      kb += BK;
      if (kb == p.Cg) {
        kb = 0;
        ++t_;
        if (++kw_ == p.nw) { kw_ = 0; if (++kh_ == p.nh) { kh_ = 0; ++kt_; } }
        retap();
      }
    };
    auto store_lds = [&](int buf) {
      char* A = smem + buf * TILE_BYTES;
      char* B = A + BM * BK * 2;
#pragma unroll
      for (int s = 0; s < A_SLOTS; ++s) {
        if constexpr (A_CHUNKS % NT != 0) if (tid + s * NT >= A_CHUNKS) break;
        uint4 v = ra[s];
        if constexpr (uaff != 0) {
          // packed consumer-side BN(+ReLU): 8 unpacks, 8 FMAs, 4 cvt_pk_bf16_f32, 4 v_pk_max_i16
          const float* sc = aff + ra_c + col * 8;
          const f32x4_t s0 = *reinterpret_cast<const f32x4_t*>(sc), s1 = *reinterpret_cast<const f32x4_t*>(sc + 4);
          const f32x4_t h0 = *reinterpret_cast<const f32x4_t*>(sc + p.Cg);
          const f32x4_t h1 = *reinterpret_cast<const f32x4_t*>(sc + p.Cg + 4);
          float f[8];
          unpack8(v, f);
          const float sc8[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
          const float sh8[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = __builtin_fmaf(f[e], sc8[e], sh8[e]);
          v = pack8_fast(f);
          if constexpr (uaff == 2) v = relu_e16x8(v);
          if constexpr (check) if (!((ra_valid >> s) & 1u)) v = uint4{0, 0, 0, 0};  // zero padding of the activation
        }
        *reinterpret_cast<uint4*>(A + sa[s]) = v;
      }
#pragma unroll
      for (int s = 0; s < B_SLOTS; ++s) {
        if constexpr (B_CHUNKS % NT != 0) if (tid + s * NT >= B_CHUNKS) break;
        *reinterpret_cast<uint4*>(B + sb[s]) = rb[s];
      }
    };
    const int nsteps = (p.nt * p.nh * p.nw * p.Cg) / BK;
    __syncthreads();  // affine table ready
    // LDS-DMA staging (UT bit 4, no input affine): buffer_load ... lds writes each wave's 64 x 16 B straight
    // into LDS (lane-linear: the XOR swizzle moves to the source column), skipping the VGPR round trip and
    // the ds_write_b128 pass (~79 B/clk/CU, the LDS bottleneck of register staging).  Two buffers: the DMA
    // of tile s+1 is issued right after the barrier of step s and lands during its MFMAs.
    // live = false (interleaved schedule, UT bit 6): the same instructions with out-of-range offsets (zeros land in a
    // buffer nobody reads any more), so the loop body stays one basic block the scheduler can interleave
    auto issue_dma = [&](int buf, bool live = true) {
      char* A = smem + buf * TILE_BYTES;
      char* B = A + BM * BK * 2;
      const int ta = tapA + kb;
#pragma unroll
      for (int s = 0; s < A_SLOTS; ++s) {
        const int rs = __builtin_amdgcn_readfirstlane((s * NT + 64 * wid) / CPR);
        if constexpr (check) {
          const bool v = live && ((tmask[s] >> t_) & 1u);
          dma16(xr, A + rs * BK * 2, v ? a_vo[s] + ta * 2 : (int)OOB, 0);
        } else {
          dma16(xr, A + rs * BK * 2, live ? a_vo[s] : (int)OOB, live ? (ta - tmin) * 2 : 0);
        }
      }
      const int wso = (tapW + kb) * 2;
#pragma unroll
      for (int s = 0; s < B_SLOTS; ++s) {
        if constexpr (B_CHUNKS % NT != 0)
          if (s * NT + 64 * wid >= B_CHUNKS) break;   // wave-uniform (B_CHUNKS is a multiple of 64)
        const int rs = __builtin_amdgcn_readfirstlane((s * NT + 64 * wid) / CPR);
        dma16(wr, B + rs * BK * 2, live ? b_vo[s] : (int)OOB, live ? wso : 0);
      }
      // branch-free cursor advance (uniform selects): keeps the loop body one scheduling region
      kb += BK;
      const int wrap = kb == p.Cg;
      kb = wrap ? 0 : kb;
      t_ += wrap;
      kw_ += wrap;
      const int wh = kw_ == p.nw;
      kw_ = wh ? 0 : kw_;
      kh_ += wh;
      const int wt = kh_ == p.nh;
      kh_ = wt ? 0 : kh_;
      kt_ += wt;
      retap();
    };
    auto issue_touch = [&]() {   // rows of the tile at the cursor (the one after the tile just issued)
      if constexpr (touch) {
        char* dst = smem + MAIN_BYTES + RED_FLOATS * 4 + (EPI >= 1 ? 6 * BN * 4 : 0) + wid * 256;
        const int ta = tapA + kb;
        // every lane issues (lanes without a row read out of range): no exec branch in the loop body
#if defined(__HIP_DEVICE_COMPILE__)
        if constexpr (check) {
          const bool v = t_on && ((t_msk >> t_) & 1u);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)dst, 4,
                                                   v ? t_vo + ta * 2 : (int)OOB, 0, 0, 0);
        } else {
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)dst, 4,
                                                   t_on ? t_vo : (int)OOB, t_on ? (ta - tmin) * 2 : 0, 0, 0);
        }
#endif
      }
    };
    constexpr int NTOUCH_DMA = touch ? 1 : 0;   // touches younger than the DMA a 2-buffer wait needs
    constexpr int NTOUCH_RING = touch ? NSTAGE - 1 : 0;   // ... than the DMA a ring wait needs
    // DMA instructions of one tile issued by this wave (A slots always; B slots only for waves whose rows exist)
    int nb_w = 0;
#pragma unroll
    for (int s = 0; s < B_SLOTS; ++s) nb_w += (s * NT + 64 * wid < B_CHUNKS) ? 1 : 0;
    nb_w = __builtin_amdgcn_readfirstlane(nb_w);
    if constexpr (glds_ut) {
      issue_dma(0);
      issue_touch();
#pragma unroll
      for (int i = 1; i + 1 < NSTAGE; ++i) {
        if (nsteps > i) issue_dma(i);
        issue_touch();
      }
    } else {
      // register ring one stage ahead of LDS: tile s+1 is written right after the barrier that frees its
      // buffer, and tile s+2 is re-issued immediately, so each load has a full k-step of MFMA to land
      load();
      store_lds(0);
      if (nsteps > 1) load();
    }
    if constexpr (glds_ut && NSTAGE == 2 && BK == 64) {
      // 2 buffers x 2 MFMA k-steps, software-pipelined across the barrier: the barrier sits between the two
      // k-steps of a tile, where (a) this tile's second-half fragments are already in registers, so every read
      // of the tile is done and its buffer can take the DMA of tile step+2, and (b) tile step+1 has landed, so
      // its first-half fragments are read while the second-half MFMAs of this tile run.  No k-step starts on
      // fragments still in flight; only barrier skew is exposed.
      ev8_t fa0[TM], fb0[TN], fa1[TM], fb1[TN];
      vm_wait<NTOUCH_DMA>();
      __syncthreads();   // tile 0 landed
      if (nsteps > 1) issue_dma(1);
      issue_touch();
#pragma unroll
      for (int i = 0; i < TM; ++i) fa0[i] = *reinterpret_cast<const ev8_t*>(smem + fa[0][i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb0[j] = *reinterpret_cast<const ev8_t*>(smem + fb[0][j]);
#pragma unroll
      for (int i = 0; i < TM; ++i) fa1[i] = *reinterpret_cast<const ev8_t*>(smem + fa[1][i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb1[j] = *reinterpret_cast<const ev8_t*>(smem + fb[1][j]);
      for (int step = 0; step < nsteps; ++step) {
        const int cur = step & 1;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = PVA_MFMA16(fb0[j], fa0[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        vm_wait<NTOUCH_DMA>();   // this wave's DMA of tile step+1
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of tile step
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const bool more = step + 1 < nsteps;
        const char* An = smem + (cur ^ 1) * TILE_BYTES;
        if constexpr ((UT >> 6) & 1) {
          // UT bit 6: the DMA issue (9 VMEM) and the next tile's first-half fragment reads (12 DS) are interleaved
          // with this tile's second-half MFMAs instead of preceding them: the two waves of a SIMD then cover each
          // other's issue with MFMA work, where the plain form leaves the matrix pipe idle while both issue DMAs
          // right after the barrier.  Branch-free (dead DMAs / reads at the tail are harmless) so the body is one
          // scheduling region.
          issue_dma(cur, step + 2 < nsteps);
          issue_touch();
#pragma unroll
          for (int i = 0; i < TM; ++i) fa0[i] = *reinterpret_cast<const ev8_t*>(An + fa[0][i]);
#pragma unroll
          for (int j = 0; j < TN; ++j) fb0[j] = *reinterpret_cast<const ev8_t*>(An + fb[0][j]);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = PVA_MFMA16(fb1[j], fa1[i], acc[i][j], 0, 0, 0);
#pragma unroll
          for (int r = 0; r < (TM * TN) / 4; ++r) {
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // one VMEM (LDS-DMA) read
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // two DS reads
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // four MFMAs
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < TM; ++i) fa1[i] = *reinterpret_cast<const ev8_t*>(An + fa[1][i]);
#pragma unroll
          for (int j = 0; j < TN; ++j) fb1[j] = *reinterpret_cast<const ev8_t*>(An + fb[1][j]);
          continue;
        }
        if (step + 2 < nsteps) issue_dma(cur);
        issue_touch();
        if (more) {
#pragma unroll
          for (int i = 0; i < TM; ++i) fa0[i] = *reinterpret_cast<const ev8_t*>(An + fa[0][i]);
#pragma unroll
          for (int j = 0; j < TN; ++j) fb0[j] = *reinterpret_cast<const ev8_t*>(An + fb[0][j]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = PVA_MFMA16(fb1[j], fa1[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (more) {
#pragma unroll
          for (int i = 0; i < TM; ++i) fa1[i] = *reinterpret_cast<const ev8_t*>(An + fa[1][i]);
#pragma unroll
          for (int j = 0; j < TN; ++j) fb1[j] = *reinterpret_cast<const ev8_t*>(An + fb[1][j]);
        }
      }
    } else
    for (int step = 0; step < nsteps; ++step) {
      const int cur = step & 1;
      const char* A;
      if constexpr (glds_ut && NSTAGE >= 3) {
        // NSTAGE-buffer ring: tiles step+1 .. step+NSTAGE-2 stay in flight across this barrier (counted vmcnt,
        // raw s_barrier — __syncthreads would drain the pending LDS-DMA with vmcnt(0)); buffer
        // (step+NSTAGE-1)%NSTAGE held tile step-1, whose readers all passed this barrier
        if (NSTAGE == 4 && step + 2 < nsteps) {
          vm_wait_dyn<2 * A_SLOTS + NTOUCH_RING, 2 * B_SLOTS>(2 * nb_w);   // leave the DMAs of tiles step+1, step+2
        } else if (step + 1 < nsteps) {
          vm_wait_dyn<A_SLOTS + NTOUCH_RING, B_SLOTS>(nb_w);   // leave this wave's A_SLOTS + nb_w DMAs of tile step+1
        } else {
          vm_wait<NTOUCH_RING>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (step + NSTAGE - 1 < nsteps) issue_dma((step + NSTAGE - 1) % NSTAGE);
        issue_touch();
        A = smem + (step % NSTAGE) * TILE_BYTES;
      } else if constexpr (glds_ut) {
        // 2 buffers (large tiles): tile step landed -> barrier -> DMA of tile step+1 during this step's MFMAs
        vm_wait<0>();
        __syncthreads();
        if (step + 1 < nsteps) issue_dma(cur ^ 1);
        A = smem + cur * TILE_BYTES;
      } else {
        __syncthreads();
        if (step + 1 < nsteps) {
          store_lds(cur ^ 1);
          if (step + 2 < nsteps) load();
        }
        A = smem + cur * TILE_BYTES;
      }
      if constexpr (glds_ut) {   // no register staging ring: room for the fragment double buffer
        mma_ktile<BK, TM, TN>(A, fa, fb, acc);
      } else {
#pragma unroll
        for (int kk = 0; kk < BK / 32; ++kk) {
          ev8_t af[TM], bfr[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const ev8_t*>(A + fa[kk][i]);
#pragma unroll
          for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const ev8_t*>(A + fb[kk][j]);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = PVA_MFMA16(bfr[j], af[i], acc[i][j], 0, 0, 0);
        }
      }
    }
  } else {
  // ---- per-slot row coordinates (fixed over the K loop) ----
    // Everything loop-invariant is precomputed here so the k-loop issues ~1 VALU op per global load:
    // a chunk's element offset = a_off[s] (row origin) + tap_lin (thread-uniform per k-step) + kc.
    const int col = tid % CPR;
    const int GHW = p.Gh * p.Gw, GTHW = p.Gt * GHW;
    const bool check = p.check != 0;   // host: false when every gathered coordinate is in range
    int a_off[A_SLOTS], a_t[A_SLOTS], a_h[A_SLOTS], a_w[A_SLOTS], sa[A_SLOTS];
    unsigned rowok = 0;
  #pragma unroll
    for (int s = 0; s < A_SLOTS; ++s) {
      const int idx = tid + s * NT;
      const int row = idx / CPR;
      const int m = m0 + row;
      a_off[s] = 0; a_t[s] = 0; a_h[s] = 0; a_w[s] = 0;
      if (idx < A_CHUNKS && m < p.M) {
        const int b = pva_fdiv(m, p.mg_thw, p.sh_thw);
        int r = m - b * RTHW;
        const int qt = pva_fdiv(r, p.mg_hw, p.sh_hw); r -= qt * RHW;
        const int qh = pva_fdiv(r, p.mg_w, p.sh_w); const int qw = r - qh * p.Rw;
        a_t[s] = qt * p.ast + p.aot; a_h[s] = qh * p.ash + p.aoh; a_w[s] = qw * p.asw + p.aow;
        a_off[s] = (b * GTHW + (a_t[s] * p.Gh + a_h[s]) * p.Gw + a_w[s]) * p.ldx;
        rowok |= 1u << s;
      }
      if constexpr (CH == 8) sa[s] = lds_off<BK>(row, col);
      else sa[s] = lds_off<BK>(row, col >> 1) + (col & 1) * 8;
    }
    int b_off[B_SLOTS], sb[B_SLOTS];
    unsigned nok = 0;
  #pragma unroll
    for (int s = 0; s < B_SLOTS; ++s) {
      const int idx = tid + s * NT;
      const int row = idx / CPR;
      const int n = n0 + row;
      b_off[s] = n * p.Kfull;
      if (idx < B_CHUNKS && n < p.Ngemm) nok |= 1u << s;
      if constexpr (CH == 8) sb[s] = lds_off<BK>(row, col);
      else sb[s] = lds_off<BK>(row, col >> 1) + (col & 1) * 8;
    }
  
    // ---- k-state of this thread's column: (channel offset, tap), with derived gather/weight offsets ----
    int kc = col * CH, kdt = 0, kdh = 0, kdw = 0;
    int tap_lin = 0, tap_w = 0;
    auto retap = [&]() {
      tap_lin = p.dir * ((kdt * p.Gh + kdh) * p.Gw + kdw) * p.ldx;
      tap_w = (((p.bt0 + kdt * p.bts) * p.kh + (p.bh0 + kdh * p.bhs)) * p.kw + (p.bw0 + kdw * p.bws)) * p.Cg;
    };
    auto kadvance = [&](int by) {
      kc += by;
      if (kc >= p.Cg) {
        do {
          kc -= p.Cg;
          if (++kdw == p.nw) { kdw = 0; if (++kdh == p.nh) { kdh = 0; ++kdt; } }
        } while (kc >= p.Cg);
        retap();
      }
    };
    retap();
    kadvance(0);
  
    VT ra[A_SLOTS], rb[B_SLOTS];
    int ra_c = 0;            // channel offset of the staged A chunks
    unsigned ra_valid = 0;   // bit s: slot s loaded real data
  
    auto load = [&]() {
      const bool tap_ok = kdt < p.nt;
      ra_c = kc; ra_valid = 0;
      const int dgt = p.dir * kdt, dgh = p.dir * kdh, dgw = p.dir * kdw;
  #pragma unroll
      for (int s = 0; s < A_SLOTS; ++s) {
        // non-short-circuit '&': three compares and ANDs instead of a branch per term
        bool v = tap_ok & ((rowok >> s & 1) != 0);
        if (check)
          v = v & ((unsigned)(a_t[s] + dgt) < (unsigned)p.Gt) & ((unsigned)(a_h[s] + dgh) < (unsigned)p.Gh) &
              ((unsigned)(a_w[s] + dgw) < (unsigned)p.Gw);
        // branch-free: an invalid slot loads from the tensor's first chunk and store_lds masks it to zero
        ra[s] = *reinterpret_cast<const VT*>(p.x + (v ? a_off[s] + tap_lin + kc : 0));
        ra_valid |= (unsigned)v << s;
      }
      const int boff = tap_w + kc;
  #pragma unroll
      for (int s = 0; s < B_SLOTS; ++s) {
        if (tap_ok && (nok >> s & 1))
          rb[s] = *reinterpret_cast<const VT*>(p.w + (b_off[s] + boff));
        else
          rb[s] = VT{};
      }
      kadvance(BK);
    };
  
    auto store_lds = [&](int buf) {
      char* A = smem + buf * TILE_BYTES;
      char* B = A + BM * BK * 2;
      // every A slot of this thread stages the same channels (ra_c): read their affine once, not once per slot
      float asc[CH], ash[CH];
      if (affine) {
  #pragma unroll
        for (int e = 0; e < CH; ++e) { asc[e] = aff[ra_c + e]; ash[e] = aff[p.Cg + ra_c + e]; }
      }
      // branch-free packed BN(+ReLU), as in the uniform-tap loader: FMAs, cvt_pk, then one v_pk_max_i16 per pair
      // against a wave-uniform floor (0 = ReLU, int16 min = none) and a mask that zeroes padding slots
      const uint32_t rfloor = affine == 2 ? 0u : 0x80008000u;
  #pragma unroll
      for (int s = 0; s < A_SLOTS; ++s) {
        if constexpr (A_CHUNKS % NT != 0) if (tid + s * NT >= A_CHUNKS) break;
        VT v = ra[s];
        const uint32_t keep = 0u - ((ra_valid >> s) & 1u);
        if (!affine) {
          if constexpr (CH == 8) v = make_uint4(v.x & keep, v.y & keep, v.z & keep, v.w & keep);
          else v = make_uint2(v.x & keep, v.y & keep);
        } else {
          float f[CH];
          if constexpr (CH == 8) unpack8(v, f); else unpack4(v, f);
  #pragma unroll
          for (int e = 0; e < CH; ++e) f[e] = __builtin_fmaf(f[e], asc[e], ash[e]);
          if constexpr (CH == 8) {
            v = pack8_fast(f);
            v = make_uint4(max_e16x2(v.x, rfloor) & keep, max_e16x2(v.y, rfloor) & keep,
                           max_e16x2(v.z, rfloor) & keep, max_e16x2(v.w, rfloor) & keep);
          } else {
            v = make_uint2(max_e16x2(cvt_pk_e16(f[0], f[1]), rfloor) & keep,
                           max_e16x2(cvt_pk_e16(f[2], f[3]), rfloor) & keep);
          }
        }
        *reinterpret_cast<VT*>(A + sa[s]) = v;
      }
  #pragma unroll
      for (int s = 0; s < B_SLOTS; ++s) {
        if constexpr (B_CHUNKS % NT != 0) if (tid + s * NT >= B_CHUNKS) break;
        *reinterpret_cast<VT*>(B + sb[s]) = rb[s];
      }
    };
  
  
    const int nsteps = (p.nt * p.nh * p.nw * p.Cg + BK - 1) / BK;
    __syncthreads();  // affine table ready
    load();
    store_lds(0);
    if (nsteps > 1) load();

    for (int step = 0; step < nsteps; ++step) {   // same one-stage-ahead register ring as above
      const int cur = step & 1;
      __syncthreads();
      if (step + 1 < nsteps) {
        store_lds(cur ^ 1);
        if (step + 2 < nsteps) load();
      }
      const char* A = smem + cur * TILE_BYTES;
  #pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        ev8_t af[TM], bfr[TN];
  #pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const ev8_t*>(A + fa[kk][i]);
  #pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const ev8_t*>(A + fb[kk][j]);
  #pragma unroll
        for (int i = 0; i < TM; ++i)
  #pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = PVA_MFMA16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    }
  }
  if constexpr ((UT >> 5) & 3) vm_wait<0>();   // touch-prefetch / dead tail DMAs still landing in LDS
  if constexpr (EPI >= 1) __syncthreads();   // the fp32 staging below overwrites the k tiles

  // ---- epilogue: D[n][m] fragment: lane holds channels n..n+3 of position m ----
  // EPI 0: direct fragment stores, cs = sum y, cq = sum y^2 (forward BN statistics)
  // EPI 1: fp32 tile staged through LDS, then the row-contiguous backward-BN pass below
  float cs[TN][4], cq[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { cs[j][r] = 0.f; cq[j][r] = 0.f; }

  const bool dense_rows = p.ost == 1 && p.osh == 1 && p.osw == 1 && p.Rt == p.Ot && p.Rh == p.Oh && p.Rw == p.Ow;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * WM + i * 16 + frow;
    int pos = m;
    if (!dense_rows && m < p.M) {
      const int b = pva_fdiv(m, p.mg_thw, p.sh_thw);
      int r = m - b * RTHW;
      const int qt = pva_fdiv(r, p.mg_hw, p.sh_hw); r -= qt * RHW;
      const int qh = pva_fdiv(r, p.mg_w, p.sh_w); const int qw = r - qh * p.Rw;
      pos = ((b * p.Ot + qt * p.ost + p.ort) * p.Oh + qh * p.osh + p.orh) * p.Ow + qw * p.osw + p.orw;
    }
    if constexpr (EPI == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WN + j * 16 + 4 * fslot;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (p.fres) {
          // residual-unit output from known BN statistics: out = relu(v*osc + osh + r), ReLU bits
          const bool ok = m < p.M && n < p.Ngemm;
          unsigned bits = 0;
          if (ok) {
            const f32x4_t sc = *reinterpret_cast<const f32x4_t*>(p.fsc + n);
            const f32x4_t sh = *reinterpret_cast<const f32x4_t*>(p.fsh + n);
            float r[4];
            unpack4(*reinterpret_cast<const uint2*>(p.eres + pos * p.ldr + n), r);
            if (p.rsc) {
              const f32x4_t rs = *reinterpret_cast<const f32x4_t*>(p.rsc + n);
              const f32x4_t rh = *reinterpret_cast<const f32x4_t*>(p.rsh + n);
#pragma unroll
              for (int e = 0; e < 4; ++e) r[e] = r[e] * rs[e] + rh[e];
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e] * sc[e] + sh[e] + r[e], 0.f);
            const uint2 pk = pack4(v);
            *reinterpret_cast<uint2*>(p.y + pos * p.ldy + n) = pk;
            const uint32_t w2[2] = {pk.x, pk.y};
#pragma unroll
            for (int e = 0; e < 2; ++e) {   // bit = stored bf16 > 0 (res_out's convention)
              bits |= ((w2[e] & 0x7fffu) != 0 && !(w2[e] & 0x8000u)) ? 1u << (2 * e) : 0u;
              bits |= ((w2[e] & 0x7fff0000u) != 0 && !(w2[e] & 0x80000000u)) ? 1u << (2 * e + 1) : 0u;
            }
          }
          // channels 8k..8k+7 of a row live in lanes l (fslot even) and l ^ 16: one mask byte per pair
          const unsigned other = swap_partner16(bits);
          if (ok && !(fslot & 1)) p.emask_out[pos * (p.Ngemm >> 3) + (n >> 3)] = (uint8_t)(bits | (other << 4));
          continue;
        }
        if (m < p.M && n < p.Ngemm) {
          uint16_t* dst = p.y + pos * p.ldy + n;
          if (p.ebias) {   // per-column bias, added in fp32 before the bf16 rounding
            const f32x4_t b = *reinterpret_cast<const f32x4_t*>(p.ebias + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += b[r];
          }
          if (p.accum) {
            float o[4];
            unpack4(*reinterpret_cast<const uint2*>(dst), o);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += o[r];
          }
          const uint2 pk = pack4(v);
          if (!p.nostore) *reinterpret_cast<uint2*>(dst) = pk;
          if (do_stats) {
            float q[4];
            unpack4(pk, q);
#pragma unroll
            for (int r = 0; r < 4; ++r) { cs[j][r] += q[r]; cq[j][r] += q[r] * q[r]; }
          }
        }
      }
    }
  }
  if constexpr (EPI >= 1) {
    // EPI 2 = the lean form (residual and / or ReLU bits and sum v only: no accumulate, no BN inputs, no bias —
    // the identity unit's conv_a dgrad after a folded conv_c): fewer registers per row, so a whole slice's rows
    // are in flight at once (one memory round trip per slice instead of two)
    // row-contiguous pass: each thread owns 8 consecutive channels (16-B global accesses) of every
    // RPP-th tile row: + old y, + residual, ReLU bits, store, backward-BN partial sums.  The fp32 tile is
    // staged through LDS (the k tiles are dead: the main loop ended with a barrier) in slices of SR rows.
    constexpr int CPRW = BN / 8, RPP = NT / CPRW;
    constexpr int SR = epi_rows(BM, BN);
    static_assert(NT % CPRW == 0, "rows per pass");
    static_assert(SR % 16 == 0 && SR % RPP == 0, "staging slices hold whole fragments and row passes");
    const int cg = tid % CPRW, r0 = tid / CPRW;
    const int n = n0 + cg * 8;
    // sv = sum v, s0 = sum v*y0, s1 = sum v*y1 ; rebased to sum v*xhat at the end of the tile
    float sv[8], s0[8], s1[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { sv[e] = 0.f; s0[e] = 0.f; s1[e] = 0.f; }
    const bool nok = n < p.Ngemm;
    const bool dual = EPI == 1 && p.ey1 != nullptr;
    const bool masky = EPI == 1 && do_bstats && p.emsc != nullptr;
    // rows whose loads are issued together (latency hiding); 2 for the 256x256 tile, whose 128 accumulator
    // registers per lane leave no room for more
    constexpr int RB = (EPI == 2 || BM * BN <= 128 * 128) ? 4 : 2;
#pragma unroll   // compile-time slices: accumulators of staged slices are dead afterwards
    for (int r_lo = 0; r_lo < BM; r_lo += SR) {
    if (r_lo > 0) __syncthreads();   // the previous slice has been read
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WM + i * 16 + frow;
      if (row < r_lo || row >= r_lo + SR) continue;   // uniform per fragment (16-row granularity)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WN + j * 16 + 4 * fslot;
        *reinterpret_cast<f32x4_t*>(smem + (row - r_lo) * STG_PITCH + col * 4) = acc[i][j];
      }
    }
    __syncthreads();
    for (int base = r_lo + r0; base < r_lo + SR && nok; base += RB * RPP) {
      uint4 lo[RB], lr[RB], l0[RB], l1[RB];
      unsigned bits[RB];
      int pos[RB];
      bool ok[RB];
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        const int rr = base + u * RPP;
        const int m = m0 + rr;
        ok[u] = rr < r_lo + SR && m < p.M;
        int ps = m;
        if (!dense_rows && ok[u]) {
          const int b = pva_fdiv(m, p.mg_thw, p.sh_thw);
          int r = m - b * RTHW;
          const int qt = pva_fdiv(r, p.mg_hw, p.sh_hw); r -= qt * RHW;
          const int qh = pva_fdiv(r, p.mg_w, p.sh_w); const int qw = r - qh * p.Rw;
          ps = ((b * p.Ot + qt * p.ost + p.ort) * p.Oh + qh * p.osh + p.orh) * p.Ow + qw * p.osw + p.orw;
        }
        pos[u] = ps;
        lo[u] = lr[u] = l0[u] = l1[u] = uint4{0, 0, 0, 0};
        bits[u] = 0xffu;
        if (ok[u]) {
          if (EPI == 1 && p.accum) lo[u] = *reinterpret_cast<const uint4*>(p.y + ps * p.ldy + n);
          if (p.eres) lr[u] = *reinterpret_cast<const uint4*>(p.eres + ps * p.ldr + n);
          if (p.emask) bits[u] = p.emask[ps * (p.Ngemm >> 3) + (n >> 3)];
          if (EPI == 1 && do_bstats) {
            if (p.ey0) l0[u] = *reinterpret_cast<const uint4*>(p.ey0 + ps * p.Ngemm + n);
            if (dual) l1[u] = *reinterpret_cast<const uint4*>(p.ey1 + ps * p.Ngemm + n);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        if (!ok[u]) continue;
        const int rr = base + u * RPP - r_lo;
        const f32x4_t va = *reinterpret_cast<const f32x4_t*>(smem + rr * STG_PITCH + cg * 32);
        const f32x4_t vb = *reinterpret_cast<const f32x4_t*>(smem + rr * STG_PITCH + cg * 32 + 16);
        float v[8] = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
        float o[8], rs[8];
        unpack8(lo[u], o);
        unpack8(lr[u], rs);
        if (masky) {  // mask mode 2: ReLU of this BN's own affine output
          float a[8];
          unpack8(l0[u], a);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (!(a[e] * bnp[4 * BN + cg * 8 + e] + bnp[5 * BN + cg * 8 + e] > 0.f)) bits[u] &= ~(1u << e);
        }
        if (EPI == 1 && p.ebias) {
          const f32x4_t b0 = *reinterpret_cast<const f32x4_t*>(p.ebias + n);
          const f32x4_t b1 = *reinterpret_cast<const f32x4_t*>(p.ebias + n + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) { rs[e] += b0[e]; rs[e + 4] += b1[e]; }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float t = v[e] + o[e] + rs[e];
          v[e] = (bits[u] >> e) & 1u ? t : 0.f;
        }
        const uint4 pk = pack8(v);
        *reinterpret_cast<uint4*>(p.y + pos[u] * p.ldy + n) = pk;
        if (do_bstats) {
          float q[8], a[8];
          unpack8(pk, q);
          unpack8(l0[u], a);   // zeros when there is no y0 (then s0 stays 0: bnp mean0/rstd0 are 0 too)
#pragma unroll
          for (int e = 0; e < 8; ++e) { sv[e] += q[e]; s0[e] += q[e] * a[e]; }
          if (dual) {
            unpack8(l1[u], a);
#pragma unroll
            for (int e = 0; e < 8; ++e) s1[e] += q[e] * a[e];
          }
        }
      }
    }
    }   // staging slices
    if (do_bstats && nok) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = cg * 8 + e;
        s0[e] = (s0[e] - bnp[c] * sv[e]) * bnp[BN + c];
        s1[e] = (s1[e] - bnp[2 * BN + c] * sv[e]) * bnp[3 * BN + c];
      }
    }
    if (do_bstats) {
      // lanes with the same channel group first reduce across the wave, then one LDS atomic per wave
      static_assert(CPRW <= 64 && (CPRW & (CPRW - 1)) == 0, "channel groups per row");
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sv[e] = wave_sum_stride(sv[e], CPRW);
        s0[e] = wave_sum_stride(s0[e], CPRW);
        s1[e] = wave_sum_stride(s1[e], CPRW);
      }
      if (lane < CPRW) {
        float* slot = red + wid * 3 * BN;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          slot[cg * 8 + e] = sv[e];
          slot[BN + cg * 8 + e] = s0[e];
          slot[2 * BN + cg * 8 + e] = s1[e];
        }
      }
      __syncthreads();
      for (int i = tid; i < BN; i += NT) {
        const int nn = n0 + i;
        if (nn < p.Ngemm) {
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            float t = 0.f;
#pragma unroll
            for (int w = 0; w < NWAVES; ++w) t += red[(w * 3 + k) * BN + i];
            p.epart[(tile_m * 3 + k) * p.Ngemm + nn] = t;
          }
        }
      }
    }
    return;
  }
  if (do_stats) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s = sum16(cs[j][r]);
        const float q = sum16(cq[j][r]);
        if (frow == 0) {  // (wm, column) slots are written by exactly one lane
          const int nl = wn * WN + j * 16 + 4 * fslot + r;
          red[wm * 2 * BN + nl] = s;
          red[wm * 2 * BN + BN + nl] = q;
        }
      }
    // raw barrier: __syncthreads would first drain every output store of the tile (vmcnt(0)) and expose
    // the write-acknowledge latency on every workgroup; only the LDS slots must be visible here
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int i = tid; i < BN; i += NT) {
      const int n = n0 + i;
      if (n < p.Ngemm) {
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int w = 0; w < BM / WM; ++w) { s += red[w * 2 * BN + i]; q += red[w * 2 * BN + BN + i]; }
        p.stats[(tile_m * 2) * p.Ngemm + n] = s;
        p.stats[(tile_m * 2 + 1) * p.Ngemm + n] = q;
      }
    }
  }
}

#ifndef PVA_KERNEL_ONLY   // (tools/gemm_lab.hip instantiates the kernel template alone)
// uniform-tap loader use: 0 never, 1 where it measured faster (default), 2 whenever legal
static int g_ut_mode = 1;

inline bool conv_ut_legal(const ConvParams& p, int ch, int bk) {
  return ch == 8 && p.Cg % bk == 0 && p.nt * p.nh * p.nw <= 32;
}

template <int BM, int BN, int WM, int WN, int CH, int BK>
void launch_cfg(const ConvParams& p, int ut_force, hipStream_t stream, bool dma = false, bool pf = false) {
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  const int m_tiles = (p.M + BM - 1) / BM, n_tiles = (p.Ngemm + BN - 1) / BN;
  const bool epi = !p.fres && (p.eres || p.emask || p.epart);   // EPI 1 (the fres epilogue is EPI 0)
  constexpr int NW = (BM / WM) * (BN / WN);
  const size_t red_bytes = epi ? (NW * 3 + 6) * BN * 4 : (BM / WM) * 2 * BN * 4;
  const bool use_dma = CH == 8 && dma && !p.affine && conv_ut_legal(p, CH, BK) && ut_force != 0;
  // touch-prefetch (cfg bit 12, UT bit 5) with the interleaved issue schedule (UT bit 6): the 2-buffer BK=64 LDS-DMA
  // loop of the big tiles only (tools/gemm_lab.hip: +9..33 % over the plain DMA loop at the res4/res5 shapes); 256 B
  // of dummy LDS per wave where the input-affine table would be (the DMA loader never has one)
  constexpr bool PF_OK = BM * BN >= 256 * 128 && BK == 64 && CH == 8;
  const bool use_pf = PF_OK && pf && use_dma;
  const size_t lds = main_lds_bytes(BM, BN, BK, epi ? 1 : 0, dma_stages(BM, BN, BK, use_dma)) + red_bytes +
                     (p.affine ? 2 * p.Cg * 4 : 0) + (use_pf ? NW * 256 : 0);
  const dim3 grid(m_tiles * n_tiles), block(NT);
  // heuristic (ut_force < 0), measured with scripts/conv_bench.py --ut 0/1/2: the uniform-tap loader wins
  // without reachable padding and for spatial (1,k,k) unit-stride gathers (with the consumer-side BN fold
  // 3x3 conv_b -20..25 %); it loses on padded temporal (k,1,1) and strided gathers.  The autotuner
  // (models/fused.ConvTuner) passes ut_force = 0 / 1 per conv instead.
  const bool ut_legal = conv_ut_legal(p, CH, BK);
  const bool ut_pays = !p.check || (p.nt == 1 && p.ash == 1 && p.asw == 1);
  const bool ut = ut_legal && (ut_force >= 0 ? ut_force == 1 : (g_ut_mode == 2 || (g_ut_mode == 1 && ut_pays)));
  // 256x256 tile (8 waves): the EPI 1 epilogue stages its fp32 tile in 64-row slices
  constexpr bool BIG = BM * BN > 128 * 128;
  if constexpr (BIG) {
    if (epi) {   // dgrad epilogue: never an input affine; the tuner only proposes the uniform-tap loader here
      // lean epilogue (EPI 2): residual / ReLU bits / sum v only
      const bool lean = !p.accum && !p.ey0 && !p.ey1 && !p.emsc && !p.ebias;
      if (lean && ut) {
        if (dma && use_pf) {
          if constexpr (PF_OK) {
            if (p.check) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 2, 115>), grid, block, lds, stream, p);
            else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 2, 113>), grid, block, lds, stream, p);
          }
        } else if (dma) {
          if (p.check) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 2, 19>), grid, block, lds, stream, p);
          else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 2, 17>), grid, block, lds, stream, p);
        } else {
          if (p.check) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 2, 3>), grid, block, lds, stream, p);
          else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 2, 1>), grid, block, lds, stream, p);
        }
        return;
      }
      if (ut && dma && use_pf) {
        if constexpr (PF_OK) {
          if (p.check) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 1, 115>), grid, block, lds, stream, p);
          else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 1, 113>), grid, block, lds, stream, p);
        }
      } else if (ut && dma) {
        if (p.check) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 1, 19>), grid, block, lds, stream, p);
        else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 1, 17>), grid, block, lds, stream, p);
      } else if (ut && p.check) {
        hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 1, 3>), grid, block, lds, stream, p);
      } else if (ut) {
        hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 1, 1>), grid, block, lds, stream, p);
      } else {
        hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 1, 0>), grid, block, lds, stream, p);
      }
      return;
    }
    if (ut && dma && !p.affine && use_pf) {
      if constexpr (PF_OK) {
        if (p.check) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 115>), grid, block, lds, stream, p);
        else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 113>), grid, block, lds, stream, p);
      }
    } else if (ut && dma && !p.affine) {
      if (p.check) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 19>), grid, block, lds, stream, p);
      else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 17>), grid, block, lds, stream, p);
    } else if (ut) {
      switch ((p.check ? 2 : 0) | (p.affine << 2)) {
        case 0: hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 1>), grid, block, lds, stream, p); break;
        case 2: hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 3>), grid, block, lds, stream, p); break;
        case 4: hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 5>), grid, block, lds, stream, p); break;
        case 6: hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 7>), grid, block, lds, stream, p); break;
        case 8: hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 9>), grid, block, lds, stream, p); break;
        default: hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 11>), grid, block, lds, stream, p); break;
      }
    } else {
      hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 0>), grid, block, lds, stream, p);
    }
    return;
  } else if constexpr (CH == 8) {
    if (ut && dma && !p.affine) {   // LDS-DMA staged uniform-tap loader (UT word bit 4)
      if (epi) {
        if (p.check) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 1, 19>), grid, block, lds, stream, p);
        else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 1, 17>), grid, block, lds, stream, p);
      } else {
        if (p.check) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 19>), grid, block, lds, stream, p);
        else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 17>), grid, block, lds, stream, p);
      }
      return;
    }
    if (epi) {   // dgrad epilogue: never an input affine
      if (ut && p.check) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 1, 3>), grid, block, lds, stream, p);
      else if (ut) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 1, 1>), grid, block, lds, stream, p);
      else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 1, 0>), grid, block, lds, stream, p);
    } else if (ut) {
      // UT word = 1 | check << 1 | affine << 2 (compile-time loader variants)
      switch ((p.check ? 2 : 0) | (p.affine << 2)) {
        case 0: hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 1>), grid, block, lds, stream, p); break;
        case 2: hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 3>), grid, block, lds, stream, p); break;
        case 4: hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 5>), grid, block, lds, stream, p); break;
        case 6: hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 7>), grid, block, lds, stream, p); break;
        case 8: hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 9>), grid, block, lds, stream, p); break;
        default: hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 11>), grid, block, lds, stream, p); break;
      }
    } else {
      hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 0>), grid, block, lds, stream, p);
    }
  } else {
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CH, BK, 0, 0>), grid, block, lds, stream, p);
  }
}

template <int CH, int BK>
void launch_variant(int v, const ConvParams& p, int ut_force, hipStream_t stream, bool dma = false, bool pf = false) {
  switch (v) {
    case 0: launch_cfg<128, 128, 64, 64, CH, BK>(p, ut_force, stream, dma); break;
    case 1: launch_cfg<128, 64, 64, 32, CH, BK>(p, ut_force, stream, dma); break;
    case 2: launch_cfg<256, 32, 64, 32, CH, BK>(p, ut_force, stream, dma); break;
    case 4:
      if constexpr (CH == 8) launch_cfg<256, 256, 128, 64, CH, BK>(p, ut_force, stream, dma, pf);
      break;
    case 5:   // 256x128 of 4 waves (128x64 each, as the 256x256 tile's): two independent workgroups per CU
      if constexpr (CH == 8) launch_cfg<256, 128, 128, 64, CH, BK>(p, ut_force, stream, dma, pf);
      break;
    default: launch_cfg<256, 16, 64, 16, CH, BK>(p, ut_force, stream, dma); break;
  }
}

#endif  // PVA_KERNEL_ONLY
}  // namespace

#ifndef PVA_KERNEL_ONLY
static int pick_variant(int M, int N) {
  if (N > 64) return 0;       // 128 x 128
  if (N > 32) return 1;       // 128 x 64
  if (N > 16) return 2;       // 256 x 32
  return 3;                   // 256 x 16
}

// Launch configuration word: tile variant (bits 0-1: 128x128, 128x64, 256x32, 256x16), BK (bit 2: 32 / 64),
// uniform-tap loader (bit 3), bit 4 set = explicit (else the built-in heuristic), bit 5 = the narrow
// direct-to-register kernel of conv_direct.hip (bit 6: 2048 rows per workgroup, else 512), bit 7 = LDS-DMA
// staging of the uniform-tap loader (launches without an input affine), bit 8 = 256x256 tile of 8 waves
// (bit 0 with it: the 256x128 tile of 4 waves instead; overrides the tile bits; bit 12 with it and BK=64 LDS-DMA: L2
// touch-prefetch of the A rows one k-tile ahead).  -1 = heuristic.
int conv_direct_rows(int cfg);
void conv_direct_launch(const ConvParams& p, int cfg, hipStream_t s);
// bit 9 = the streaming pointwise kernel of conv_pw.hip (dense 1x1x1 GEMMs; bits 0-1: 1024 << v rows per
// workgroup)
int conv_pw_rows(int cfg);
int conv_pw_legal(const ConvParams& p, int chunk);
void conv_pw_launch(const ConvParams& p, int cfg, hipStream_t st);
// bit 11 = the halo-staged (1,3,3) kernel of conv_halo.hip (bit 0: 64-channel n-tiles; bits 12+: positions per
// tile, which is its BN partial-sum row tile)
void conv_halo_launch(const ConvParams& p, int cfg, hipStream_t st);

int conv_cfg_bm(int cfg, int N) {
  if (cfg >= 0 && (cfg & 16) && (cfg & 2048)) return cfg >> 12;
  if (cfg >= 0 && (cfg & 16) && (cfg & 512)) return conv_pw_rows(cfg);
  if (cfg >= 0 && (cfg & 16) && (cfg & 32)) return conv_direct_rows(cfg);
  if (cfg >= 0 && (cfg & 16) && (cfg & 256)) return 256;   // 256x256 tile
  const int v = (cfg >= 0 && (cfg & 16)) ? (cfg & 3) : pick_variant(0, N);
  return v <= 1 ? 128 : 256;
}

int conv_igemm_m_tiles(int M, int N) {
  const int bm = conv_cfg_bm(-1, N);
  return (M + bm - 1) / bm;
}

int conv_igemm_m_tiles_k(int M, int N, int /*K*/, int /*Cg*/) { return conv_igemm_m_tiles(M, N); }

static int g_bk_override = -1;
void conv_igemm_set_ut(int mode) { g_ut_mode = mode; }
void conv_igemm_set_bk(int bk) { g_bk_override = bk; }

// 1 when the uniform-tap loader may run this launch with that BK
int conv_igemm_ut_legal(const ConvParams& p, int chunk, int bk) { return conv_ut_legal(p, chunk, bk) ? 1 : 0; }

void conv_igemm_launch(const ConvParams& p0, int chunk, hipStream_t stream, int cfg) {
  if ((p0.eres || p0.emask || p0.epart || p0.fres) && chunk != 8) return;  // host binding rejects this combination
  ConvParams p = p0;
  pva_magic_div(p.Rt * p.Rh * p.Rw, &p.mg_thw, &p.sh_thw);
  pva_magic_div(p.Rh * p.Rw, &p.mg_hw, &p.sh_hw);
  pva_magic_div(p.Rw, &p.mg_w, &p.sh_w);
  int v, bk, ut_force;
  bool dma = false, pf = false;
  if (cfg >= 0 && (cfg & 16) && (cfg & 2048)) {  // halo-staged 3x3 kernel (legality checked by the bindings)
    conv_halo_launch(p, cfg, stream);
    return;
  }
  if (cfg >= 0 && (cfg & 16) && (cfg & 512)) {   // streaming pointwise kernel (legality checked by the bindings)
    conv_pw_launch(p, cfg, stream);
    return;
  }
  if ((p.fres || p.ebias || p.nostore) && cfg >= 0 && (cfg & 32)) cfg = -1;   // direct kernel: no fres / bias / nostore
  if (cfg >= 0 && (cfg & 16) && (cfg & 32)) {  // narrow direct-to-register kernel (conv_direct.hip)
    conv_direct_launch(p, cfg, stream);
    return;
  }
  if (cfg >= 0 && (cfg & 16)) {
    v = (cfg & 256) ? 4 + (cfg & 1) : (cfg & 3);
    bk = (cfg & 4) ? 64 : 32;
    ut_force = (cfg >> 3) & 1;
    dma = (cfg & 128) != 0;   // LDS-DMA staging (uniform-tap loader, no input affine)
    pf = (cfg & 256) && (cfg & 4096);   // big tiles, BK=64 LDS-DMA: L2 touch-prefetch one k-tile ahead
  } else {
    v = pick_variant(p.M, p.Ngemm);
    const int K = p.nt * p.nh * p.nw * p.Cg;
    bk = g_bk_override > 0 ? g_bk_override : ((K >= 1024 && chunk == 8) ? 64 : 32);
    ut_force = -1;
  }
  if (chunk == 8) {
    if (bk == 64) launch_variant<8, 64>(v, p, ut_force, stream, dma, pf); else launch_variant<8, 32>(v, p, ut_force, stream, dma);
  } else {
    if (bk == 64) launch_variant<4, 64>(v, p, ut_force, stream); else launch_variant<4, 32>(v, p, ut_force, stream);
  }
}

#endif  // PVA_KERNEL_ONLY

PVA_NS_END  // namespace PVA_NS
