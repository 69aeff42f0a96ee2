// Direct (halo-tiled) space-to-depth stem convolutions for SlowFast / Slow on gfx950.
//
// The stems are 7x7 stride-2 convs on 3-channel frames (slow: k(1,7,7), Cout 64; fast: k(5,7,7),
// Cout 8).  As implicit GEMMs they are hopeless: Cout 8 leaves MFMA columns idle and each input pixel is
// re-gathered ~60x through the cache hierarchy (the fast stem alone was 12 % of a training step).
// Instead:
//   * the preprocessing kernel writes stem inputs in space-to-depth layout: a 2x2 pixel block x RGB0 =
//     16 bf16 channels, so the conv becomes k(kt,4,4) stride 1 with 32-byte positions (weights for
//     the tap positions outside the 7x7 window are zero);
//   * a workgroup owns an 8x16 output tile of one clip and walks its frames: input frames live in an
//     LDS ring (each frame is read from HBM exactly once per tile); the next frame (and, for wgrad, the
//     next dY tile) is copied by LDS-DMA (buffer_load ... lds) while the current one computes, so no
//     VGPRs or ds_writes are spent on staging; one barrier per frame;
//   * forward: all weight fragments sit in VGPRs (A operand), input fragments are one ds_read_b128
//     each (B operand), BN partial sums are produced in the epilogue;
//   * wgrad: dY tile of the frame is staged in LDS, both MFMA operands are read with the gfx950
//     transpose read ds_read_b64_tr_b16 (positions are the reduction axis), each wave keeps a slice of
//     the taps in accumulators across all frames, and adds it to the fp32 dW accumulator once.
#include "common.h"
#include <stdlib.h>
#include <string.h>
#include <cstdlib>

PVA_NS_BEGIN

namespace {

constexpr int TH = 8, TW = 16;              // output tile (positions = 128 = 4 waves x 2 rows)
constexpr int PH = TH + 3, PW = TW + 3;     // s2d patch (kernel 4)
constexpr int POSB = 32;                    // bytes per s2d position (16 bf16)

struct StemParams {
  const uint16_t* x;    // [N, T, Hs, Ws, 16] s2d input
  const uint16_t* w;    // forward: [Cout_pad][taps*16] packed s2d weights
  uint16_t* y;          // [N, To, Ho, Wo, Cout]
  float* stats;         // [nblocks][2][Cout]
  const uint16_t* dy;   // wgrad: [N, To, Ho, Wo, Cout]
  float* dw;            // wgrad accumulator [Cout][taps*16] fp32
  int N, T, Hs, Ws, Cout;
  int To, Ho, Wo;
  int pt;               // temporal padding (kt/2)
  int tiles_h, tiles_w;
  int slab;             // wgrad: 0 = fp32 atomics into dw; else each workgroup stores its partial dW to dw + block * slab
};                      //        (reproducible mode: fixed-order reduction by stem_slab_reduce)

constexpr uint32_t OOB = 0x7ffffff0u;         // buffer offset past num_records: the load returns zeros
constexpr int SLOT_BYTES = 448 * 16;           // frame slot: 418 chunks padded to 7 x 64 lanes

// 16-B LDS-DMA of one lane: buffer_load_dwordx4 ... lds into wave-uniform LDS address `lds` + 16 * lane
// (the address_space(3) cast only exists in the device pass)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, (int)voff, 0, 0, 0);
#endif
}

// LDS position swizzle of the wgrad kernels' 32-byte-position images: bit 2 of the position flips with bit 3.
// Their transpose reads fetch positions p..p+3 (lanes 0-15) and p+8..p+11 (lanes 16-31) in one 32-lane bank
// group; unswizzled, positions 8 apart (256 B) hit the same banks (2-way conflict on every read, brute-force
// checked); swizzled, the two quads cover all 64 banks.  An involution within aligned 16-position groups.
__device__ __forceinline__ int pswz(int pos) { return pos ^ ((pos >> 1) & 4); }

// one input frame's s2d patch -> LDS slot by LDS-DMA; positions outside the frame / image read zeros
// through out-of-range buffer offsets.  No VGPR staging, no ds_write: the copy overlaps the MFMA loop.
// SWZ: LDS position k holds patch position pswz(k) (the DMA stays lane-linear; the swizzle moves to the source).
template <bool SWZ = false>
__device__ __forceinline__ void dma_patch(__amdgpu_buffer_rsrc_t r, const StemParams& p, int ti, int hs0, int ws0,
                                          char* slot) {
  const int tid = threadIdx.x, w = tid >> 6;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (s == 1 && w == 3) break;  // chunks 448.. do not exist (wave-uniform)
    const int idx = tid + s * 256;
    const int pos = SWZ ? pswz(idx >> 1) : (idx >> 1), half = idx & 1;
    const int r_ = pos / PW, c_ = pos - r_ * PW;
    const int hs = hs0 + r_ - 2, ws = ws0 + c_ - 2;
    const bool ok = pos < PH * PW && ti >= 0 && ti < p.T && (unsigned)hs < (unsigned)p.Hs &&
                    (unsigned)ws < (unsigned)p.Ws;
    const uint32_t vo = ok ? (uint32_t)((((ti * p.Hs + hs) * p.Ws + ws) * 16 + half * 8) * 2) : OOB;
    dma16(r, slot + (w * 64 + s * 256) * 16, vo);  // chunks 418..447 land in the slot padding
  }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t clip_rsrc(const uint16_t* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

// ------------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------------
// PERM (Cout == 16 COT, COT even): the A fragment rows of block pair (2m, 2m+1) are permuted so that a lane ends with
// 8 consecutive channels of its position (row r of block 2m+h = channel 32m + 8(r>>2) + 4h + (r&3)): one 16-B store
// per block pair instead of two 8-B stores, a position's 128-B row written by 2 instructions of 64-B pieces (the
// slow stem writes 2 GB per step)
template <int KT, int COT, bool PERM = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void stem_fwd_kernel(const StemParams p) {
  constexpr int TAPS = KT * 16;
  constexpr int KSTEPS = TAPS * 16 / 32;  // 2 taps per MFMA k-step
  constexpr int SLOTS = KT + 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem + SLOTS * SLOT_BYTES);  // [4 waves][2][COT*16]

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  // XCD-aware tile order: consecutive tiles (horizontal neighbours, then rows) on one XCD, so the halo rows/columns a
  // tile shares with its neighbours come from that XCD's L2 (blockIdx order spread them over all 8: 1.75x the input
  // bytes from HBM, profiles/r5_pmc)
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int b = L;
  const int tw = b % p.tiles_w; b /= p.tiles_w;
  const int th = b % p.tiles_h;
  const int n = b / p.tiles_h;
  const int ho0 = th * TH, wo0 = tw * TW;

  const __amdgpu_buffer_rsrc_t xr =
      clip_rsrc(p.x + (int64_t)n * p.T * p.Hs * p.Ws * 16, (uint32_t)(p.T * p.Hs * p.Ws * 32));
  // weight fragments (A operand: lane holds W[co = 16*c + li][k = 32*ks + 8*g .. +8])
  ev8_t wa[COT][KSTEPS];
  auto chan = [&](int c, int r) { return PERM ? 32 * (c >> 1) + 8 * (r >> 2) + 4 * (c & 1) + (r & 3) : 16 * c + r; };
#pragma unroll
  for (int c = 0; c < COT; ++c)
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks)
      wa[c][ks] = *reinterpret_cast<const ev8_t*>(p.w + (int64_t)chan(c, li) * (TAPS * 16) + ks * 32 + 8 * g);

  // prologue: frames -pt .. -pt+KT-1 into slots 0..KT-1 (frame ti lives in slot (ti + pt) % SLOTS)
  for (int f = 0; f < KT; ++f) dma_patch(xr, p, f - p.pt, ho0, wo0, smem + f * SLOT_BYTES);
  __syncthreads();

  float cs[COT][4], cq[COT][4];
#pragma unroll
  for (int c = 0; c < COT; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) { cs[c][r] = 0.f; cq[c][r] = 0.f; }

  const int ww = li;                 // position column inside the tile
  const int half = g & 1;            // channel half of the lane's 8 k-values
  for (int to = 0; to < p.To; ++to) {
    if (to + 1 < p.To)  // frame needed first by the next output frame, into the slot outside the window
      dma_patch(xr, p, to - p.pt + KT, ho0, wo0, smem + ((to + KT) % SLOTS) * SLOT_BYTES);
    f32x4_t acc[2][COT];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int c = 0; c < COT; ++c) acc[q][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      const int tap = 2 * ks + (g >> 1);
      const int dt = tap >> 4, bh = (tap >> 2) & 3, bw = tap & 3;
      const char* slot = smem + ((to + dt) % SLOTS) * SLOT_BYTES;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int hh = 2 * w + q;
        const ev8_t xb = *reinterpret_cast<const ev8_t*>(
            slot + ((hh + bh) * PW + (ww + bw)) * POSB + half * 16);
#pragma unroll
        for (int c = 0; c < COT; ++c)
          acc[q][c] = PVA_MFMA16(wa[c][ks], xb, acc[q][c], 0, 0, 0);
      }
    }
    __syncthreads();  // next frame landed; window frame 0's slot is free.  Stores after the barrier.
    // epilogue: D[co][pos]: lane holds co = chan(c, 4g + r) for position (row 2w+q, col li)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ho = ho0 + 2 * w + q, wo = wo0 + li;
      const bool valid = ho < p.Ho && wo < p.Wo;
      const int64_t pos = (((int64_t)n * p.To + to) * p.Ho + ho) * p.Wo + wo;
      if constexpr (PERM) {
#pragma unroll
        for (int m = 0; m < COT / 2; ++m) {
          if (valid) {
            float v[8] = {acc[q][2 * m][0], acc[q][2 * m][1], acc[q][2 * m][2], acc[q][2 * m][3],
                          acc[q][2 * m + 1][0], acc[q][2 * m + 1][1], acc[q][2 * m + 1][2], acc[q][2 * m + 1][3]};
            const uint4 pk = pack8(v);
            *reinterpret_cast<uint4*>(p.y + pos * p.Cout + 32 * m + 8 * g) = pk;
            float f[8];
            unpack8(pk, f);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              cs[2 * m][r] += f[r]; cq[2 * m][r] += f[r] * f[r];
              cs[2 * m + 1][r] += f[4 + r]; cq[2 * m + 1][r] += f[4 + r] * f[4 + r];
            }
          }
        }
        continue;
      }
#pragma unroll
      for (int c = 0; c < COT; ++c) {
        const int co = 16 * c + 4 * g;
        if (valid && co < p.Cout) {
          float v[4] = {acc[q][c][0], acc[q][c][1], acc[q][c][2], acc[q][c][3]};
          const uint2 pk = pack4(v);
          *reinterpret_cast<uint2*>(p.y + pos * p.Cout + co) = pk;
          float f[4];
          unpack4(pk, f);
#pragma unroll
          for (int r = 0; r < 4; ++r) { cs[c][r] += f[r]; cq[c][r] += f[r] * f[r]; }
        }
      }
    }
  }
  // BN partial sums of this workgroup: one slot per wave, summed in wave order (deterministic)
  constexpr int CT = COT * 16;
#pragma unroll
  for (int c = 0; c < COT; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s = sum16(cs[c][r]), q = sum16(cq[c][r]);
      if (li == 0) {
        red[w * 2 * CT + chan(c, 4 * g + r)] = s;
        red[w * 2 * CT + CT + chan(c, 4 * g + r)] = q;
      }
    }
  __syncthreads();
  for (int i = tid; i < p.Cout; i += 256) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) { s += red[k * 2 * CT + i]; q += red[k * 2 * CT + CT + i]; }
    p.stats[(int64_t)L * 2 * p.Cout + i] = s;
    p.stats[(int64_t)L * 2 * p.Cout + p.Cout + i] = q;
  }
}

// ------------------------------------------------------------------------------------------------
// weight gradient
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ s16x4_t trr(const char* a) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(a));
}

// The same transpose read as inline asm: the compiler's wait-count pass treats the intrinsic as possibly reading the
// LDS an in-flight LDS-DMA writes and puts an s_waitcnt vmcnt(0) in front of it — right after the next frame pair's
// DMAs are issued, so no DMA overlapped the MFMAs (the barrier at the end of the pair already waits for them).  The
// asm form is invisible to that pass: its results are made ready by explicit lgkmcnt waits (lgkm_tie) that also carry
// the registers, so nothing consumes them earlier.
__device__ __forceinline__ s16x4_t trr_nw(const char* a) {
  s16x4_t r;
  const uint32_t off = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)a);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(off));
  return r;
}

// s_waitcnt lgkmcnt(N) that the four registers depend on.  LDS reads retire in order, so after the wait every LDS
// read older than the N newest is complete, whatever other lgkm operations are in flight.
template <int N>
__device__ __forceinline__ void lgkm_tie(s16x4_t& a, s16x4_t& b, s16x4_t& c, s16x4_t& d) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N));
}

__device__ __forceinline__ ev8_t frag8(s16x4_t lo, s16x4_t hi) {
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(ev8_t, v);
}

// AR: transpose reads through trr_nw, the reads of k-step k + 1 requested before the MFMAs of k-step k (see trr_nw)
template <int KT, int COT, bool AR = false>
__global__ __launch_bounds__(256) void stem_wgrad_kernel(const StemParams p) {
  constexpr int TAPS = KT * 16;
  constexpr int TPW = TAPS / 4;              // taps per wave
  constexpr int SLOTS = KT + 1;
  constexpr int COP = COT * 16;
  constexpr int DYB = TH * TW * COP * 2;     // dY tile bytes [128 pos][COP co]
  constexpr int DYC = TH * TW * COP / 8 / 256;  // 16-B dY chunks per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* dyt = smem + SLOTS * SLOT_BYTES;     // two dY tile buffers (frame parity)

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  // XCD-aware tile order: consecutive tiles (horizontal neighbours, then rows) on one XCD, so the halo rows/columns a
  // tile shares with its neighbours come from that XCD's L2 (blockIdx order spread them over all 8: 1.75x the input
  // bytes from HBM, profiles/r5_pmc)
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int b = L;
  const int tw = b % p.tiles_w; b /= p.tiles_w;
  const int th = b % p.tiles_h;
  const int n = b / p.tiles_h;
  const int ho0 = th * TH, wo0 = tw * TW;
  const __amdgpu_buffer_rsrc_t xr =
      clip_rsrc(p.x + (int64_t)n * p.T * p.Hs * p.Ws * 16, (uint32_t)(p.T * p.Hs * p.Ws * 32));
  const __amdgpu_buffer_rsrc_t yr = clip_rsrc(p.dy + (int64_t)n * p.To * p.Ho * p.Wo * p.Cout,
                                              (uint32_t)(p.To * p.Ho * p.Wo * p.Cout * 2));
  // dY tile of frame `to` -> buf by LDS-DMA: chunk idx = pos * (COP / 8) + ch / 8 at LDS offset idx * 16
  auto dma_dy = [&](int to, char* buf) {
#pragma unroll
    for (int k = 0; k < DYC; ++k) {
      const int idx = tid + k * 256;
      const int pos = idx / (COP / 8), ch = (idx % (COP / 8)) * 8;
      const int ho = ho0 + pos / TW, wo = wo0 + pos % TW;
      const bool ok = ho < p.Ho && wo < p.Wo && ch < p.Cout;
      const uint32_t vo = ok ? (uint32_t)((((to * p.Ho + ho) * p.Wo + wo) * p.Cout + ch) * 2) : OOB;
      dma16(yr, buf + (k * 256 + w * 64) * 16, vo);
    }
  };

  f32x4_t acc[COT][TPW];
#pragma unroll
  for (int c = 0; c < COT; ++c)
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[c][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int f = 0; f < KT; ++f) dma_patch(xr, p, f - p.pt, ho0, wo0, smem + f * SLOT_BYTES);
  dma_dy(0, dyt);
  __syncthreads();
  // tr-read lane roles: group g covers positions 8g..8g+7 of a 32-position k-step (rows of 16 w);
  // lane supplies row (li >> 2) of a 4-row block and 4 columns at 8*(li & 3) bytes.
  const int rq = li >> 2, cb = (li & 3) * 8;
  for (int to = 0; to < p.To; ++to) {
    const char* dcur = dyt + (to & 1) * DYB;
    if (to + 1 < p.To) {  // next frame's input (slot outside the window) and dY tile (other buffer)
      dma_patch(xr, p, to - p.pt + KT, ho0, wo0, smem + ((to + KT) % SLOTS) * SLOT_BYTES);
      dma_dy(to + 1, dyt + ((to + 1) & 1) * DYB);
    }
    if constexpr (AR) {
      constexpr int KS = TH * TW / 32, NR = COT + TPW;   // fragments per k-step: COT dY + TPW taps, 2 reads each
      static_assert(NR % 2 == 0, "ties go by 4 halves");
      s16x4_t R[2][NR][2];
      auto issue = [&](int kstep, s16x4_t (&Rk)[NR][2]) {
        const int hh = 2 * kstep + (g >> 1), wq = 8 * (g & 1) + rq;
#pragma unroll
        for (int c = 0; c < COT; ++c) {
          const char* base = dcur + (hh * TW + wq) * COP * 2 + c * 32 + cb;
          Rk[c][0] = trr_nw(base);
          Rk[c][1] = trr_nw(base + 4 * COP * 2);
        }
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          const int tap = w * TPW + t;
          const int dt = tap >> 4, bh = (tap >> 2) & 3, bw = tap & 3;
          const char* base = smem + ((to + dt) % SLOTS) * SLOT_BYTES + ((hh + bh) * PW + (wq + bw)) * POSB + cb;
          Rk[COT + t][0] = trr_nw(base);
          Rk[COT + t][1] = trr_nw(base + 4 * POSB);
        }
      };
      issue(0, R[0]);
#pragma unroll
      for (int kstep = 0; kstep < KS; ++kstep) {
        s16x4_t(&Rk)[NR][2] = R[kstep & 1];
        if (kstep + 1 < KS) {
          issue(kstep + 1, R[(kstep + 1) & 1]);
          // at most 15 reads (the counter's limit) in flight: all of this k-step's reads are older than those
#pragma unroll
          for (int i = 0; i < NR; i += 2) lgkm_tie<(2 * NR < 15 ? 2 * NR : 15)>(Rk[i][0], Rk[i][1], Rk[i + 1][0], Rk[i + 1][1]);
        } else {
#pragma unroll
          for (int i = 0; i < NR; i += 2) lgkm_tie<0>(Rk[i][0], Rk[i][1], Rk[i + 1][0], Rk[i + 1][1]);
        }
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          const ev8_t xb = frag8(Rk[COT + t][0], Rk[COT + t][1]);
#pragma unroll
          for (int c = 0; c < COT; ++c) acc[c][t] = PVA_MFMA16(frag8(Rk[c][0], Rk[c][1]), xb, acc[c][t], 0, 0, 0);
        }
      }
      __syncthreads();  // next frame + dY tile landed; the window's first slot and this dY buffer are free
      continue;
    }
#pragma unroll
    for (int kstep = 0; kstep < TH * TW / 32; ++kstep) {
      // positions of this k-step: rows 2*kstep, 2*kstep+1; group g -> row 2*kstep + (g >> 1), w 8*(g&1)..+7
      const int hh = 2 * kstep + (g >> 1);
      const int wq = 8 * (g & 1) + rq;          // position column of the lane's tr-read row (first block)
      ev8_t a[COT];
#pragma unroll
      for (int c = 0; c < COT; ++c) {
        const char* base = dcur + (hh * TW + wq) * COP * 2 + c * 32 + cb;
        s16x4_t lo = trr(base), hi = trr(base + 4 * COP * 2);
        s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        a[c] = __builtin_bit_cast(ev8_t, v);
      }
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const int tap = w * TPW + t;
        const int dt = tap >> 4, bh = (tap >> 2) & 3, bw = tap & 3;
        const char* slot = smem + ((to + dt) % SLOTS) * SLOT_BYTES;
        const char* base = slot + ((hh + bh) * PW + (wq + bw)) * POSB + cb;
        s16x4_t lo = trr(base), hi = trr(base + 4 * POSB);
        s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const ev8_t xb = __builtin_bit_cast(ev8_t, v);
#pragma unroll
        for (int c = 0; c < COT; ++c)
          acc[c][t] = PVA_MFMA16(a[c], xb, acc[c][t], 0, 0, 0);
      }
    }
    __syncthreads();  // next frame + dY tile landed; the window's first slot and this dY buffer are free
  }
  // D[co][k]: lane holds channel k = li of tap, co = 16c + 4g + r
#pragma unroll
  for (int c = 0; c < COT; ++c)
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int tap = w * TPW + t;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 16 * c + 4 * g + r;
        if (co < p.Cout) {
          const int64_t o = (int64_t)co * TAPS * 16 + tap * 16 + li;
          if (p.slab) p.dw[(int64_t)blockIdx.x * p.slab + o] = acc[c][t][r];
          else atomicAdd(p.dw + o, acc[c][t][r]);
        }
      }
    }
}

// ------------------------------------------------------------------------------------------------
// Cout == 8 temporal stem (fast pathway, k(KT,7,7)): two output frames per MFMA.
// With 8 output channels half of a 16-row MFMA tile is idle.  Here rows 0-7 carry output frame t and
// rows 8-15 frame t+1: for input frame j of the pair's window (j = f - t + pt = 0..KT) frame t uses tap
// j and frame t+1 tap j-1, so the A fragment of window frame j is [W[:, j]; W[:, j-1]] and one MFMA
// serves both frames — KT+1 input frames per output pair instead of 2*KT (40 % fewer MFMAs at KT = 5).
// The wgrad kernel mirrors it with the dY tiles of the two frames stacked as 16 "channels".
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ ev8_t ld_frag(const uint16_t* p, bool ok) {
  const uint4 u = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
  return __builtin_bit_cast(ev8_t, u);
}

template <int KT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void stem_fwd_pair_kernel(const StemParams p) {
  constexpr int TAPS = KT * 16;
  constexpr int J = KT + 1;     // input frames per output-frame pair
  constexpr int KS = 8;         // k-steps per input frame: 16 spatial taps x 16 channels / 32
  constexpr int SLOTS = J + 2;  // window frame j of pair t0 lives in slot (t0 + j) % SLOTS; +2 in flight
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem + SLOTS * SLOT_BYTES);  // [4 waves][2][8]

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  // XCD-aware tile order: consecutive tiles (horizontal neighbours, then rows) on one XCD, so the halo rows/columns a
  // tile shares with its neighbours come from that XCD's L2 (blockIdx order spread them over all 8: 1.75x the input
  // bytes from HBM, profiles/r5_pmc)
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int b = L;
  const int tw = b % p.tiles_w; b /= p.tiles_w;
  const int th = b % p.tiles_h;
  const int n = b / p.tiles_h;
  const int ho0 = th * TH, wo0 = tw * TW;
  const __amdgpu_buffer_rsrc_t xr =
      clip_rsrc(p.x + (int64_t)n * p.T * p.Hs * p.Ws * 16, (uint32_t)(p.T * p.Hs * p.Ws * 32));

  for (int f = 0; f < J; ++f) dma_patch(xr, p, f - p.pt, ho0, wo0, smem + f * SLOT_BYTES);

  ev8_t wa[J][KS];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int dt = li < 8 ? j : j - 1;
    const bool ok = dt >= 0 && dt < KT;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wa[j][ks] = ld_frag(p.w + (int64_t)(li & 7) * (TAPS * 16) + (ok ? dt : 0) * 256 + ks * 32 + 8 * g, ok);
  }
  __syncthreads();  // drains this wave's DMAs (vmcnt(0)) and publishes every wave's

  float cs[4] = {0.f, 0.f, 0.f, 0.f}, cq[4] = {0.f, 0.f, 0.f, 0.f};
  const int half = g & 1;
  const int co0 = 4 * (g & 1);  // D rows 4g..4g+3: channels co0.. of output frame t0 + (g >> 1)
  for (int t0 = 0; t0 < p.To; t0 += 2) {
    if (t0 + 2 < p.To) {  // the next pair's two new frames, into slots outside the current window
      const int tn = t0 - p.pt + J;
      dma_patch(xr, p, tn, ho0, wo0, smem + ((t0 + J) % SLOTS) * SLOT_BYTES);
      dma_patch(xr, p, tn + 1, ho0, wo0, smem + ((t0 + J + 1) % SLOTS) * SLOT_BYTES);
    }
    f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const char* slot = smem + ((t0 + j) % SLOTS) * SLOT_BYTES;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int tap = 2 * ks + (g >> 1);
        const int bh = tap >> 2, bw = tap & 3;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const ev8_t xb = *reinterpret_cast<const ev8_t*>(
              slot + ((2 * w + q + bh) * PW + (li + bw)) * POSB + half * 16);
          acc[q] = PVA_MFMA16(wa[j][ks], xb, acc[q], 0, 0, 0);
        }
      }
    }
    // barrier first (next frames landed; window frames 0, 1 free), then this pair's stores: their write
    // latency hides behind the next pair's MFMAs instead of stalling at a barrier
    __syncthreads();
    const int to = t0 + (g >> 1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ho = ho0 + 2 * w + q, wo = wo0 + li;
      if (ho < p.Ho && wo < p.Wo && to < p.To) {
        const int64_t pos = (((int64_t)n * p.To + to) * p.Ho + ho) * p.Wo + wo;
        float v[4] = {acc[q][0], acc[q][1], acc[q][2], acc[q][3]};
        const uint2 pk = pack4(v);
        *reinterpret_cast<uint2*>(p.y + pos * 8 + co0) = pk;
        float f[4];
        unpack4(pk, f);
#pragma unroll
        for (int r = 0; r < 4; ++r) { cs[r] += f[r]; cq[r] += f[r] * f[r]; }
      }
    }
  }
  // BN partial sums: lanes g and g^2 hold the same channels (frames t0 / t0+1); fixed summation order
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float s = sum16(cs[r]), q = sum16(cq[r]);
    s += __shfl_xor(s, 32, 64);
    q += __shfl_xor(q, 32, 64);
    if (li == 0 && g < 2) {
      red[w * 16 + 4 * g + r] = s;
      red[w * 16 + 8 + 4 * g + r] = q;
    }
  }
  __syncthreads();
  if (tid < 8) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) { s += red[k * 16 + tid]; q += red[k * 16 + 8 + tid]; }
    p.stats[(int64_t)L * 16 + tid] = s;
    p.stats[(int64_t)L * 16 + 8 + tid] = q;
  }
}

// ROLL (default): wave w owns spatial tap column bw = w and walks the four tap rows bh in registers.  The B fragment of
// (kstep k, bh + 2) is the one of (k + 1, bh) (two output rows per kstep), so each kstep reads two new input fragments
// instead of four and a window frame's 16 MFMAs cost 5 fragment reads instead of 16; the dY fragments of the four
// ksteps are read once per frame pair.  Without it (arm stem_roll=0) wave w owns tap row bh = w and reads every
// fragment per MFMA: 2 transpose reads per MFMA make the kernel LDS-bound (35.7 % MFMA busy, profiles/r5_final).
// AR (with ROLL, default): every transpose read through trr_nw, software-pipelined — the fragments of k-step k + 1 are
// requested before the MFMAs of k-step k — so the next pair's DMAs overlap this pair's MFMAs (arm stem_async=0: the
// intrinsic reads and the vmcnt(0) the compiler puts in front of them).
template <int KT, bool ROLL, bool AR = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void stem_wgrad_pair_kernel(const StemParams p) {
  constexpr int TAPS = KT * 16;
  constexpr int J = KT + 1;
  constexpr int SLOTS = J + 2;
  constexpr int DYB = TH * TW * 16 * 2;  // dY tile [128 pos][16]: frame t0 (0-7) | frame t0+1 (8-15)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* dyt = smem + SLOTS * SLOT_BYTES;  // two dY tile buffers (pair parity)

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  // XCD-aware tile order: consecutive tiles (horizontal neighbours, then rows) on one XCD, so the halo rows/columns a
  // tile shares with its neighbours come from that XCD's L2 (blockIdx order spread them over all 8: 1.75x the input
  // bytes from HBM, profiles/r5_pmc)
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int b = L;
  const int tw = b % p.tiles_w; b /= p.tiles_w;
  const int th = b % p.tiles_h;
  const int n = b / p.tiles_h;
  const int ho0 = th * TH, wo0 = tw * TW;
  const __amdgpu_buffer_rsrc_t xr =
      clip_rsrc(p.x + (int64_t)n * p.T * p.Hs * p.Ws * 16, (uint32_t)(p.T * p.Hs * p.Ws * 32));
  const __amdgpu_buffer_rsrc_t yr =
      clip_rsrc(p.dy + (int64_t)n * p.To * p.Ho * p.Wo * 8, (uint32_t)(p.To * p.Ho * p.Wo * 16));
  // dY chunk of this lane: position tid >> 1 of the tile, frame t0 + (tid & 1); LDS offset tid * 16
  const int dpos = pswz(tid >> 1), dfh = tid & 1;   // swizzled dY image (see pswz)
  const int dho = ho0 + dpos / TW, dwo = wo0 + dpos % TW;
  const bool dok = dho < p.Ho && dwo < p.Wo;
  auto dma_dy = [&](int t0, char* buf) {
    const int to = t0 + dfh;
    const uint32_t vo = dok && to < p.To ? (uint32_t)((((to * p.Ho + dho) * p.Wo + dwo) * 8) * 2) : OOB;
    dma16(yr, buf + w * 64 * 16, vo);
  };

  // wave w owns spatial taps (bh = w, bw = 0..3) of every window frame: both halves of a (co, dt) sum
  // end up in the same wave (rows 0-7 of acc[dt], rows 8-15 of acc[dt+1]) and are combined by a shuffle.
  f32x4_t acc[J][4];
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int s = 0; s < 4; ++s) acc[j][s] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int f = 0; f < J; ++f) dma_patch<true>(xr, p, f - p.pt, ho0, wo0, smem + f * SLOT_BYTES);
  dma_dy(0, dyt);
  __syncthreads();
  const int rq = li >> 2, cb = (li & 3) * 8;
  for (int t0 = 0; t0 < p.To; t0 += 2) {
    const char* dcur = dyt + ((t0 >> 1) & 1) * DYB;
    if (t0 + 2 < p.To) {
      const int tn = t0 - p.pt + J;
      dma_patch<true>(xr, p, tn, ho0, wo0, smem + ((t0 + J) % SLOTS) * SLOT_BYTES);
      dma_patch<true>(xr, p, tn + 1, ho0, wo0, smem + ((t0 + J + 1) % SLOTS) * SLOT_BYTES);
      dma_dy(t0 + 2, dyt + (((t0 >> 1) + 1) & 1) * DYB);
    }
    if constexpr (ROLL && AR) {
      constexpr int KS = TH * TW / 32;
      const int h0 = g >> 1, wq = 8 * (g & 1) + rq;
      ev8_t af[KS];
      {
        s16x4_t al[KS], ah[KS];
#pragma unroll
        for (int kstep = 0; kstep < KS; ++kstep) {
          const int dp = (2 * kstep + h0) * TW + wq;
          al[kstep] = trr_nw(dcur + pswz(dp) * 32 + cb);
          ah[kstep] = trr_nw(dcur + pswz(dp + 4) * 32 + cb);
        }
        lgkm_tie<0>(al[0], ah[0], al[1], ah[1]);
        lgkm_tie<0>(al[2], ah[2], al[3], ah[3]);
#pragma unroll
        for (int kstep = 0; kstep < KS; ++kstep) af[kstep] = frag8(al[kstep], ah[kstep]);
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const char* slot = smem + ((t0 + j) % SLOTS) * SLOT_BYTES;
        // F[m]: patch rows 2m + h0 (even fragment: halves 0, 1) and 2m + h0 + 1 (odd: halves 2, 3), tap column w;
        // k-step k uses F[k] (tap rows 0, 1) and F[k + 1] (tap rows 2, 3)
        s16x4_t F[KS + 1][4];
        auto issue = [&](int m) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int ip = (2 * m + h0 + e) * PW + wq + w;
            F[m][2 * e] = trr_nw(slot + pswz(ip) * POSB + cb);
            F[m][2 * e + 1] = trr_nw(slot + pswz(ip + 4) * POSB + cb);
          }
        };
        issue(0);
        issue(1);
#pragma unroll
        for (int kstep = 0; kstep < KS; ++kstep) {
          if (kstep + 2 <= KS) {
            issue(kstep + 2);   // in flight during this k-step's MFMAs
            if (kstep == 0) lgkm_tie<4>(F[0][0], F[0][1], F[0][2], F[0][3]);
            lgkm_tie<4>(F[kstep + 1][0], F[kstep + 1][1], F[kstep + 1][2], F[kstep + 1][3]);
          } else {
            lgkm_tie<0>(F[kstep + 1][0], F[kstep + 1][1], F[kstep + 1][2], F[kstep + 1][3]);
          }
          acc[j][0] = PVA_MFMA16(af[kstep], frag8(F[kstep][0], F[kstep][1]), acc[j][0], 0, 0, 0);
          acc[j][1] = PVA_MFMA16(af[kstep], frag8(F[kstep][2], F[kstep][3]), acc[j][1], 0, 0, 0);
          acc[j][2] = PVA_MFMA16(af[kstep], frag8(F[kstep + 1][0], F[kstep + 1][1]), acc[j][2], 0, 0, 0);
          acc[j][3] = PVA_MFMA16(af[kstep], frag8(F[kstep + 1][2], F[kstep + 1][3]), acc[j][3], 0, 0, 0);
        }
      }
      __syncthreads();  // next frames / dY tile landed; current window frames 0, 1 and dY buffer are free
      continue;
    }
    if constexpr (ROLL) {
      constexpr int KS = TH * TW / 32;
      const int h0 = g >> 1, wq = 8 * (g & 1) + rq;
      ev8_t af[KS];
#pragma unroll
      for (int kstep = 0; kstep < KS; ++kstep) {
        const int dp = (2 * kstep + h0) * TW + wq;
        s16x4_t lo = trr(dcur + pswz(dp) * 32 + cb), hi = trr(dcur + pswz(dp + 4) * 32 + cb);
        s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[kstep] = __builtin_bit_cast(ev8_t, v);
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const char* slot = smem + ((t0 + j) % SLOTS) * SLOT_BYTES;
        auto frag = [&](int row) {   // patch row `row` (per lane), tap column w
          const int ip = row * PW + wq + w;
          s16x4_t lo = trr(slot + pswz(ip) * POSB + cb), hi = trr(slot + pswz(ip + 4) * POSB + cb);
          s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          return __builtin_bit_cast(ev8_t, v);
        };
        ev8_t fe = frag(h0), fo = frag(h0 + 1);
#pragma unroll
        for (int kstep = 0; kstep < KS; ++kstep) {
          const int hh = 2 * kstep + h0;
          const ev8_t fe2 = frag(hh + 2), fo2 = frag(hh + 3);
          acc[j][0] = PVA_MFMA16(af[kstep], fe, acc[j][0], 0, 0, 0);
          acc[j][1] = PVA_MFMA16(af[kstep], fo, acc[j][1], 0, 0, 0);
          acc[j][2] = PVA_MFMA16(af[kstep], fe2, acc[j][2], 0, 0, 0);
          acc[j][3] = PVA_MFMA16(af[kstep], fo2, acc[j][3], 0, 0, 0);
          fe = fe2;
          fo = fo2;
        }
      }
      __syncthreads();  // next frames / dY tile landed; current window frames 0, 1 and dY buffer are free
      continue;
    }
#pragma unroll
    for (int kstep = 0; kstep < TH * TW / 32; ++kstep) {
      const int hh = 2 * kstep + (g >> 1);
      const int wq = 8 * (g & 1) + rq;
      ev8_t a;
      {
        const int dp = hh * TW + wq;
        s16x4_t lo = trr(dcur + pswz(dp) * 32 + cb), hi = trr(dcur + pswz(dp + 4) * 32 + cb);
        s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        a = __builtin_bit_cast(ev8_t, v);
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const char* slot = smem + ((t0 + j) % SLOTS) * SLOT_BYTES;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int ip = (hh + w) * PW + (wq + s);
          s16x4_t lo = trr(slot + pswz(ip) * POSB + cb), hi = trr(slot + pswz(ip + 4) * POSB + cb);
          s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          acc[j][s] = PVA_MFMA16(a, __builtin_bit_cast(ev8_t, v), acc[j][s], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // next frames / dY tile landed; current window frames 0, 1 and dY buffer are free
  }
  // dW[co][dt][tap] = rows 0-7 of acc[dt] (lanes g < 2) + rows 8-15 of acc[dt + 1] (lanes g >= 2)
#pragma unroll
  for (int dt = 0; dt < KT; ++dt)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = g < 2 ? acc[dt][s][r] : acc[dt + 1][s][r];
        v += __shfl_xor(v, 32, 64);
        // acc[.][s]: tap (bh = w, bw = s), or with ROLL (bh = s, bw = w)
        const int tap = ROLL ? 4 * s + w : 4 * w + s;
        if (g < 2) {
          const int64_t o = (int64_t)(4 * g + r) * TAPS * 16 + (dt * 16 + tap) * 16 + li;
          if (p.slab) p.dw[(int64_t)blockIdx.x * p.slab + o] = v;
          else atomicAdd(p.dw + o, v);
        }
      }
}

// acc[i] += sum over slabs s = 0, 1, ... of slab[s * n + i], in that order (bitwise reproducible)
__global__ __launch_bounds__(256) void stem_slab_reduce_kernel(const float* slab, int nslab, int n, float* acc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = acc[i];
  for (int k = 0; k < nslab; ++k) v += slab[(int64_t)k * n + i];
  acc[i] = v;
}

// dW (s2d accumulator [Cout][kt][4][4][sy][sx][c4]) -> grad [Cout][3][kt][7][7] ; re-zeroes the accumulator
__global__ void stem_wgrad_convert_kernel(float* __restrict__ acc, float* __restrict__ grad, int Cout, int kt,
                                          float beta) {
  const int total = Cout * 3 * kt * 49;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
    int r = o;
    const int kw = r % 7; r /= 7;
    const int kh = r % 7; r /= 7;
    const int dt = r % kt; r /= kt;
    const int c = r % 3;
    const int co = r / 3;
    const int bh = (kh + 1) >> 1, sy = (kh + 1) & 1, bw = (kw + 1) >> 1, sx = (kw + 1) & 1;
    const int a = co * kt * 256 + ((dt * 4 + bh) * 4 + bw) * 16 + (sy * 2 + sx) * 4 + c;
    grad[o] = (beta == 0.f ? 0.f : beta * grad[o]) + acc[a];
  }
}

__global__ void zero_kernel(float* p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = 0.f;
}

// fp32 [Cout][3][kt][7][7] -> bf16 s2d packed [Cout_pad16][kt*16 taps][16]
__global__ void stem_pack_kernel(const float* __restrict__ w, uint16_t* __restrict__ out, int Cout, int Cpad, int kt) {
  const int K = kt * 256;
  const int total = Cpad * K;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int co = i / K;
    int k = i % K;
    const int ch = k % 16, tap = k / 16;
    const int c = ch % 4, sx = (ch / 4) & 1, sy = ch / 8;
    const int bw = tap % 4, bh = (tap / 4) % 4, dt = tap / 16;
    const int kh = 2 * bh + sy - 1, kw = 2 * bw + sx - 1;
    float v = 0.f;
    if (co < Cout && c < 3 && kh >= 0 && kh < 7 && kw >= 0 && kw < 7)
      v = w[(((co * 3 + c) * kt + dt) * 7 + kh) * 7 + kw];
    out[i] = f2e(v);
  }
}

template <int KT, int COT, bool PERM = false>
void launch_fwd(const StemParams& p, hipStream_t s) {
  const size_t lds = (KT + 1) * SLOT_BYTES + 4 * 2 * COT * 16 * 4;
  hipLaunchKernelGGL((stem_fwd_kernel<KT, COT, PERM>), dim3(p.N * p.tiles_h * p.tiles_w), dim3(256), lds, s, p);
}

template <int KT, int COT, bool AR = false>
void launch_wgrad(const StemParams& p, hipStream_t s) {
  const size_t lds = (KT + 1) * SLOT_BYTES + 2 * TH * TW * COT * 16 * 2;
  hipLaunchKernelGGL((stem_wgrad_kernel<KT, COT, AR>), dim3(p.N * p.tiles_h * p.tiles_w), dim3(256), lds, s, p);
}

template <int KT>
void launch_fwd_pair(const StemParams& p, hipStream_t s) {
  const size_t lds = (KT + 3) * SLOT_BYTES + 4 * 16 * 4;
  hipLaunchKernelGGL((stem_fwd_pair_kernel<KT>), dim3(p.N * p.tiles_h * p.tiles_w), dim3(256), lds, s, p);
}

template <int KT, bool ROLL, bool AR = false>
void launch_wgrad_pair(const StemParams& p, hipStream_t s) {
  const size_t lds = (KT + 3) * SLOT_BYTES + 2 * TH * TW * 16 * 2;
  hipLaunchKernelGGL((stem_wgrad_pair_kernel<KT, ROLL, AR>), dim3(p.N * p.tiles_h * p.tiles_w), dim3(256), lds, s, p);
}

}  // namespace

int stem_tiles(int Ho, int Wo, int N) { return N * ((Ho + TH - 1) / TH) * ((Wo + TW - 1) / TW); }

// Alternate arms of the stem A/Bs (pytorchvideo_accelerate_amd/utils/arms.py, one knob: PVA_ARMS="stem_pair=0,...").
// Read per launch (two launches per step) so tests can switch kernels within one process.
//   stem_pair  frame-pair kernels for Cout == 8 temporal stems (0: the one-frame kernels)
//   stem_perm  channel-permuted 16-B stores of the Cout-64 stem forward (0: the 8-B-store epilogue)
//   stem_roll  frame-pair wgrad with B fragments rolled across k-steps (0: one tap row per wave)
//   stem_async rolling wgrad with asm transpose reads + explicit lgkmcnt (0: the intrinsic reads)
static int stem_arm(const char* name) {
  const char* e = getenv("PVA_ARMS");
  if (e == nullptr) return 1;
  const size_t n = strlen(name);
  for (const char* p = strstr(e, name); p != nullptr; p = strstr(p + 1, name)) {
    const bool start = p == e || p[-1] == ',' || p[-1] == ' ';
    if (start && p[n] == '=') return atoi(p + n + 1);
  }
  return 1;
}
static bool stem_pair_enabled() { return stem_arm("stem_pair") != 0; }
static bool stem_perm_enabled() { return stem_arm("stem_perm") != 0; }
static bool stem_roll_enabled() { return stem_arm("stem_roll") != 0; }
static bool stem_async_enabled() { return stem_arm("stem_async") != 0; }

// mode 0: forward, 1: wgrad.  Shapes outside stem_s2d_supported() are rejected by the bindings (TORCH_CHECK)
// before this is reached, so every call launches exactly one kernel.
void stem_s2d_launch(int mode, const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, const uint16_t* dy,
                     float* dw, int N, int T, int Hs, int Ws, int Cout, int kt, hipStream_t s, float* slab) {
  StemParams p{};
  p.x = x; p.w = w; p.y = y; p.stats = stats; p.dy = dy; p.dw = slab != nullptr ? slab : dw;
  p.slab = slab != nullptr ? Cout * kt * 256 : 0;
  p.N = N; p.T = T; p.Hs = Hs; p.Ws = Ws; p.Cout = Cout;
  p.To = T; p.Ho = Hs; p.Wo = Ws; p.pt = kt / 2;
  p.tiles_h = (Hs + TH - 1) / TH; p.tiles_w = (Ws + TW - 1) / TW;
  const bool pair = stem_pair_enabled() && kt == 5 && Cout == 8;
  if (mode == 0) {
    if (pair) launch_fwd_pair<5>(p, s);
    else if (kt == 5 && Cout <= 16) launch_fwd<5, 1>(p, s);
    else if (kt == 1 && Cout == 64 && stem_perm_enabled()) launch_fwd<1, 4, true>(p, s);
    else if (kt == 1 && Cout <= 64) launch_fwd<1, 4>(p, s);
  } else {
    if (pair && stem_roll_enabled() && stem_async_enabled()) launch_wgrad_pair<5, true, true>(p, s);
    else if (pair && stem_roll_enabled()) launch_wgrad_pair<5, true>(p, s);
    else if (pair) launch_wgrad_pair<5, false>(p, s);
    else if (kt == 5 && Cout <= 16) launch_wgrad<5, 1>(p, s);
    else if (kt == 1 && Cout <= 64 && stem_async_enabled()) launch_wgrad<1, 4, true>(p, s);
    else if (kt == 1 && Cout <= 64) launch_wgrad<1, 4>(p, s);
    if (slab != nullptr) {   // fixed-order sum of the per-workgroup partials into the accumulator
      const int n = Cout * kt * 256, nslab = p.N * p.tiles_h * p.tiles_w;
      hipLaunchKernelGGL(stem_slab_reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, s, slab, nslab, n, dw);
    }
  }
}

bool stem_s2d_supported(int Cout, int kt) { return (kt == 5 && Cout <= 16) || (kt == 1 && Cout <= 64); }

void stem_wgrad_convert_launch(float* acc, float* grad, int Cout, int kt, float beta, hipStream_t s) {
  const int total = Cout * 3 * kt * 49;
  hipLaunchKernelGGL(stem_wgrad_convert_kernel, dim3((total + 255) / 256), dim3(256), 0, s, acc, grad, Cout, kt, beta);
  const int n = Cout * kt * 256;
  hipLaunchKernelGGL(zero_kernel, dim3((n + 255) / 256), dim3(256), 0, s, acc, n);
}

void stem_pack_launch(const float* w, uint16_t* out, int Cout, int kt, hipStream_t s) {
  const int Cpad = (Cout + 15) / 16 * 16;
  const int total = Cpad * kt * 256;
  hipLaunchKernelGGL(stem_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, s, w, out, Cout, Cpad, kt);
}

PVA_NS_END  // namespace PVA_NS
