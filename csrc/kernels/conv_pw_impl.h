// Pointwise conv kernel template and its launchers (included by the per-KS instantiation units
// conv_pw_ks{1,2,4,8}.hip, compiled in parallel; the public entry points live in conv_pw.hip).
//
// Pointwise (1x1x1, unit-stride, unpadded) convolution as a streaming GEMM on MFMA (gfx950).
//
// Why a separate kernel: the implicit-GEMM kernel (conv_igemm.hip) runs ONE output tile per workgroup.
// For a 1x1 conv with a short K (<= 256) that tile has only K/32 MFMA steps, so every tile pays the whole
// load -> MFMA -> epilogue latency chain with little to overlap it, and these memory-bound layers (the
// bottleneck's conv_a / conv_c / branch1 and their dgrads, the BN-folded residual output) ran at
// 2.3-3.6 TB/s (profiles/r2_layers).  Here:
//   * the packed weights live in LDS, pre-arranged in MFMA fragment order (each 1-KB fragment is read by
//     a wave as one contiguous, conflict-free ds_read_b128), filled once per workgroup; convs whose weights
//     exceed the LDS budget are split into output-channel groups (one workgroup per group and row range);
//   * each wave streams 16*TM-row tiles: the tile's activations are loaded ONCE into registers (the
//     producer's BatchNorm + ReLU applied on the way) and reused for every 32-channel output chunk;
//   * each chunk's epilogue operands (residual, old output, BN inputs, mask bits) are issued one or two
//     iterations ahead through a register ring, so several chunks of loads stay in flight per wave (with
//     only 8 waves per CU, a single chunk in flight capped these layers at ~3.5 TB/s by Little's law);
//   * all global traffic goes through buffer descriptors rebased per workgroup (out-of-range rows load
//     zero / drop stores in hardware: no per-row predicates), and each instantiation carries only its
//     own operand streams (OPS);
//   * per-channel epilogue constants are staged in LDS once per workgroup;
//   * output channels are permuted inside each 32-channel chunk so a lane's two accumulator fragments hold
//     8 CONSECUTIVE channels of one position: 16-B stores, 16-B residual / BN-input loads, and one
//     ReLU-mask byte per lane (no cross-lane shuffles);
//   * per-channel statistics are reduced across the 16 lanes of a fragment column by a DPP butterfly
//     reduce-scatter (15 DPP adds for 16 values), accumulated in per-wave LDS slots and summed over the
//     waves in a fixed order: one partial slab per workgroup, bitwise run-to-run deterministic.
// Epilogues (EP): 0 plain (+bias, +accumulate, +forward BN statistics), 1 the BN-folded residual-unit
// output (conv_igemm's fres), 2 the backward-BN epilogue of the dgrads (conv_igemm's EPI 1).
#pragma once
#include "common.h"
#include "conv_params.h"
#include <algorithm>

PVA_NS_BEGIN

namespace {

constexpr int PW_LDS = 156 * 1024;     // LDS budget of a workgroup (weights, statistics, constants)

// Butterfly reduce-scatter over the 16 lanes sharing lane >> 4 (one DPP row): v[L] in; lane rho ends up
// holding the 16-lane total of element rho (L = 16) or of element rho >> 1 (L = 8) in v[0].  The partners
// are DPP lane permutations (no LDS crossbar): rho ^ 8 (row_ror:8), rho ^ 7 (row_half_mirror), rho ^ 2 and
// rho ^ 1 (quad_perm) — linearly independent masks, so the four stages cover all 16 lanes; at each stage
// the lane's selector bit (3, 2, 1, 0) picks the half it keeps.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}

template <int CTRL, int BIT, int HALF, int L>
__device__ __forceinline__ void rs_stage(float (&v)[L], int lane) {
  // blend through a bit mask: a plain ?: lets the compiler turn the select into a lane-dependent array
  // index, lowered as compare/select chains over the whole array (measured: ~500 extra instructions)
  const unsigned hm = (lane >> BIT) & 1 ? 0xffffffffu : 0u;
#pragma unroll
  for (int j = 0; j < HALF; ++j) {
    const unsigned lo = __float_as_uint(v[j]), hi = __float_as_uint(v[j + HALF]);
    const unsigned x = (lo ^ hi) & hm;
    const float send = __uint_as_float(hi ^ x);   // selector set: lo, else hi
    const float keep = __uint_as_float(lo ^ x);   // selector set: hi, else lo
    v[j] = keep + dpp_f<CTRL>(send);
  }
}

constexpr int DPP_XOR8 = 0x128;   // row_ror:8
constexpr int DPP_XOR7 = 0x141;   // row_half_mirror
constexpr int DPP_XOR2 = 0x4e;    // quad_perm [2, 3, 0, 1]
constexpr int DPP_XOR1 = 0xb1;    // quad_perm [1, 0, 3, 2]

template <int L>
__device__ __forceinline__ void rs16(float (&v)[L], int lane) {
  static_assert(L == 8 || L == 16, "16 or 8 values");
  if constexpr (L == 16) {
    rs_stage<DPP_XOR8, 3, 8>(v, lane);
    rs_stage<DPP_XOR7, 2, 4>(v, lane);
    rs_stage<DPP_XOR2, 1, 2>(v, lane);
    rs_stage<DPP_XOR1, 0, 1>(v, lane);
  } else {
    rs_stage<DPP_XOR8, 3, 4>(v, lane);
    rs_stage<DPP_XOR7, 2, 2>(v, lane);
    rs_stage<DPP_XOR2, 1, 1>(v, lane);
    v[0] += dpp_f<DPP_XOR1>(v[0]);
  }
}

typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t_;

// epilogue operands of one 32-channel chunk (members an epilogue does not use are optimised away)
template <int TM>
struct Pre {
  uint4 old[TM], res[TM], y0[TM], y1[TM];
  unsigned bits[TM];
};

// OPS: the epilogue operand streams this instantiation reads (OP_OLD accumulate, OP_RES residual, OP_Y0 /
// OP_Y1 BN inputs, OP_MASK ReLU bits, OP_MSC ReLU from affine(y0)); an instantiation carries registers (and
// buffer descriptors / branches) only for its own streams, so the ring can be deeper
constexpr int OP_OLD = 1, OP_RES = 2, OP_Y0 = 4, OP_Y1 = 8, OP_MASK = 16, OP_MSC = 32;
constexpr int OP_RAFF = 64;   // EP 1: the residual goes through BN_1's affine (unit 0's branch1); else identity

// ReLU bits of 8 packed non-negative 16-bit values (bit e: element e > 0, i.e. a non-zero magnitude — the sign bit of
// a ReLU output is set only for -0): (w & 0x7fff7fff) + 0x7fff7fff carries each non-zero half into its top bit
// (bit 15 / 31) without crossing halves, then one bitfield extract per element (the compare/select chains the
// compiler made of the per-half test cost ~4.5 VALU per element in the residual-output epilogue)
__device__ __forceinline__ unsigned relu_bits8(const uint4& pk) {
  const uint32_t t0 = (pk.x & 0x7fff7fffu) + 0x7fff7fffu, t1 = (pk.y & 0x7fff7fffu) + 0x7fff7fffu;
  const uint32_t t2 = (pk.z & 0x7fff7fffu) + 0x7fff7fffu, t3 = (pk.w & 0x7fff7fffu) + 0x7fff7fffu;
  return __builtin_amdgcn_ubfe(t0, 15, 1) | (__builtin_amdgcn_ubfe(t0, 31, 1) << 1) |
         (__builtin_amdgcn_ubfe(t1, 15, 1) << 2) | (__builtin_amdgcn_ubfe(t1, 31, 1) << 3) |
         (__builtin_amdgcn_ubfe(t2, 15, 1) << 4) | (__builtin_amdgcn_ubfe(t2, 31, 1) << 5) |
         (__builtin_amdgcn_ubfe(t3, 15, 1) << 6) | (__builtin_amdgcn_ubfe(t3, 31, 1) << 7);
}

// NW: waves per workgroup — 8, or 4 (cfg bit 3: an instantiation between 128 and 168 VGPRs then runs three
// workgroups = 12 waves per CU instead of one 8-wave workgroup, the register file no longer rounding to 2 per SIMD)
template <int KS, int TM, int EP, int AFF, bool NTS, int OPS, int PD, int CPI, bool TP, int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2))) void conv_pw_kernel(const ConvParams p, int rpb, int gch) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NST = EP == 2 ? 3 : 2;
  constexpr int NSLOT = EP == 1 ? 0 : NST * NW;   // per-wave statistic slots (= conv_pw.hip)
  constexpr int MT = 16 * TM;   // PD: prefetch ring depth (chunks)
  const int N = p.Ngemm, K = p.Kfull, Ca = p.Cg;   // K = taps x Ca (1x1: K = Ca)
  // output-channel group of this workgroup (weights of wide convs do not fit LDS at once: the row range
  // is walked once per group of gch 32-channel chunks; the XCD remap puts the groups of one row range on
  // the same XCD, so its activations are re-read from that L2)
  const int ngrp = ((N >> 5) + gch - 1) / gch;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = L % ngrp, rblk = L / ngrp;
  const int cbase = grp * gch;                              // first chunk of the group
  const int nch = min(gch, (N >> 5) - cbase);               // chunks in this group
  const int NG = nch * 32, nb0 = cbase * 32;                // group channels, first channel
  const int wimg = nch * 2 * KS * 1024;
  float* st_lds = reinterpret_cast<float*>(smem + wimg);   // [NW][NST][NG] per-wave statistics
  float* cst = st_lds + NSLOT * NG;                         // [4][NG] per-channel epilogue constants
  float* affs = cst + 4 * NG;                               // [2][Ca] input affine (per gathered channel)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rho = lane & 15, g = lane >> 4;
  // this wave's statistic slots: every (statistic, channel) address is updated by one lane of one wave, in
  // tile order, and the waves' slots are summed in a fixed order at the end — run-to-run deterministic
  float* sw = st_lds + wid * NST * NG;

  // ---- weight image: fragment f = (c * 2 + h) * KS + s, lane l's 16 B at f * 1024 + 16 l:
  //      row rho of half h of chunk c = output channel 32c + 8(rho >> 2) + 4h + (rho & 3), k = 32s + 8(l >> 4)
  const int units = nch * 2 * KS * 64;
  for (int u = tid; u < units; u += (NW * 64)) {
    const int l = u & 63, f = u >> 6;
    const int s = f % KS, ch = f / KS;
    const int h = ch & 1, c = ch >> 1;
    const int r = l & 15;
    const int n = nb0 + 32 * c + 8 * (r >> 2) + 4 * h + (r & 3);
    const int k0 = 32 * s + 8 * (l >> 4);
    uint4 v = uint4{0, 0, 0, 0};
    if (k0 < K) v = *reinterpret_cast<const uint4*>(p.w + (int64_t)n * p.Kfull + k0);
    *reinterpret_cast<uint4*>(smem + (int64_t)u * 16) = v;
  }
  const bool do_stats = (EP == 0 && p.stats != nullptr) || (EP == 2 && p.epart != nullptr);
  const bool nostore = EP == 0 && p.nostore != 0;
  if (do_stats)
    for (int i = tid; i < NSLOT * NG; i += (NW * 64)) st_lds[i] = 0.f;
  if (AFF)
    for (int i = tid; i < Ca; i += (NW * 64)) { affs[i] = p.in_scale[i]; affs[Ca + i] = p.in_shift[i]; }
  // EP 1: fsc fsh rsc rsh ; EP 0 / 2: bias (0 when absent), mask-affine scale and shift
  for (int i = tid; i < NG; i += (NW * 64)) {
    const int n = nb0 + i;
    if (EP == 1) {
      cst[i] = p.fsc[n]; cst[NG + i] = p.fsh[n];
      cst[2 * NG + i] = p.rsc ? p.rsc[n] : 1.f; cst[3 * NG + i] = p.rsh ? p.rsh[n] : 0.f;
    } else {
      cst[i] = p.ebias ? p.ebias[n] : 0.f;
      if (EP == 2 && (OPS & OP_MSC)) { cst[NG + i] = p.emsc[n]; cst[2 * NG + i] = p.emsh[n]; }
    }
  }
  __syncthreads();

  const int row0 = rblk * rpb;
  const int row_end = min(p.M, row0 + rpb);
  const int nrows = row_end - row0;
  const int mrow = N >> 3;   // mask bytes per row
  constexpr bool dual = EP == 2 && (OPS & OP_Y1);   // (the launcher sets OP_Y1 only with statistics)
  constexpr bool masky = EP == 2 && (OPS & OP_MSC);
  constexpr bool need_y0 = EP == 2 && (OPS & OP_Y0);
  constexpr bool stat_b = EP == 0 || need_y0;       // second statistic: sum v^2 (EP 0) / sum v y0 (EP 2)

  // Buffer resources rebased to this workgroup's first row and sized to its rows: rows past the tensor's
  // end (its last, partial tile) load zeros and drop their stores in hardware, so no load or store
  // carries a per-row predicate (the predicated flat version spent ~25 VALU ops per output element on
  // addressing, exec masks and SGPR spills).  Offsets: per-row VGPR (row and this lane's 8 channels),
  // per-chunk SGPR.
  auto rsrc = [&](const void* base, int row_bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<const char*>(base) + (int64_t)row0 * row_bytes), (short)0, nrows * row_bytes,
        0x00020000);
  };
  const int xb = p.ldx * 2, yb = p.ldy * 2, rb = p.ldr * 2, nb = N * 2;
  const __amdgpu_buffer_rsrc_t xr = rsrc(p.x, xb);
  const __amdgpu_buffer_rsrc_t yr = rsrc(p.y, yb);
  __amdgpu_buffer_rsrc_t resr = yr, mr = yr, y0r = yr, y1r = yr, mor = yr;
  if constexpr (EP != 0 && (OPS & OP_RES)) resr = rsrc(p.eres, rb);
  if constexpr (EP == 2) {
    if constexpr ((OPS & OP_MASK) != 0) mr = rsrc(p.emask, mrow);
    if constexpr (need_y0) y0r = rsrc(p.ey0, nb);
    if constexpr (dual) y1r = rsrc(p.ey1, nb);
  }
  if constexpr (EP == 1) mor = rsrc(p.emask_out, mrow);
  constexpr int ST_AUX = NTS ? 2 : 0;   // nt (streaming) store policy bit
  // Stores take their whole offset in the VGPR (soffset 0): with an SGPR soffset the compiler assumes a
  // >8-byte store's data VGPRs may be overwritten by the very next VALU op, which corrupted lanes 12-15
  // of each row of the stored dwords on gfx950 (test_pw_fres); with soffset 0 it inserts the wait state.
  constexpr uint32_t OOB = 0x80000000u;

  // A wave walks its tiles (16*TM rows: mfirst + t * tstride) and, per tile, the chunks CPI at a time
  // (an iteration):
  //  * the epilogue operands of iteration it are issued PD - 1 iterations ahead (a register ring);
  //  * CPI = 2: a lane's two chunks are the two 64-B halves of one 128-B line of its row, read and written
  //    within one iteration — with one chunk per iteration the halves were touched ~5 us apart and
  //    measured 30 % extra DRAM traffic (lines evicted in between, scripts/gpu_r2_pwpmc.sh);
  //  * the next tile's activations are loaded (raw) when a tile starts; the producer's BN + ReLU is
  //    applied when that tile starts.  (Running the ring itself across tile boundaries cost ~55 VGPRs
  //    and spills; so did seemingly equivalent rewrites of the prefetch below — check
  //    -Rpass-analysis=kernel-resource-usage after touching it.)
  const int nit = (nch + CPI - 1) / CPI;
  const int tstride = NW * MT;
  const int mfirst = row0 + wid * MT;
  const int ntw = mfirst < row_end ? (row_end - mfirst + tstride - 1) / tstride : 0;
  // this lane's activation offsets within a row (k past K -> out of bounds -> zero).  Temporal taps (kt,1,1),
  // unit stride (fwd, or the stride-1 dgrad gathering backwards): k = 32 s + 8 g is tap j = k / Ca, channel
  // k % Ca, read from the row (t + aot + dir j) of the same clip and pixel — a whole-row delta of
  // (aot + dir j) * H * W rows; taps leaving the clip read zero (padding).  Tap rows may lie outside this
  // workgroup's row range, so they go through a resource over the whole tensor.
  constexpr bool taps = TP;   // (launch_ks: p.nt > 1)
  const int HW = p.Rh * p.Rw;
  uint32_t xk[KS];
  int kc[KS], tdel[KS], rdel[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k0 = 32 * s + 8 * g;
    const int j = k0 / Ca;
    kc[s] = k0 - j * Ca;
    tdel[s] = p.aot + p.dir * j;
    rdel[s] = tdel[s] * HW * xb;
    xk[s] = k0 < K ? (taps ? kc[s] : k0) * 2 : OOB;
  }
  const __amdgpu_buffer_rsrc_t xall = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.xbytes,
                                                                        0x00020000);
  uint4 araw[TM][KS];
  unsigned amask = 0;   // taps: (row i, chunk s) inside the clip -> bit i * KS + s
  auto load_a = [&](int m0) {
    if constexpr (taps) {
      const int q0 = m0 / HW;
      const int rem0 = m0 - q0 * HW;
      const int t0 = q0 % p.Rt;
      amask = 0;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int pos = rem0 + 16 * i + rho;   // < HW + 64 <= 3 HW (host: HW >= 32): at most two slice steps
        int tr = t0 + (pos >= HW ? 1 : 0) + (pos >= 2 * HW ? 1 : 0);
        if (tr >= p.Rt) tr -= p.Rt;
        const int base = (m0 + 16 * i + rho) * xb;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const int tt = tr + tdel[s];
          const bool v = xk[s] != OOB && tt >= 0 && tt < p.Gt;
          araw[i][s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
              xall, v ? (uint32_t)(base + rdel[s]) + xk[s] : OOB, 0, 0));
          amask |= (v ? 1u : 0u) << (i * KS + s);
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const uint32_t ro = (uint32_t)(m0 - row0 + 16 * i + rho) * xb;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        araw[i][s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, xk[s] == OOB ? OOB : ro + xk[s], 0, 0));
    }
  };
  Pre<TM> P[PD][CPI];
  bool pairbits = false;   // the current prefetch loads a chunk pair's ReLU bits with one 8-B load
  // row r's offsets (rows relative to row0; this lane's 8 channels 8g.. folded in)
  auto prefetch1 = [&](int m0, int c, Pre<TM>& Q) {
    const int nc = nb0 + 32 * c;   // chunk's first channel (uniform)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const uint32_t r = (uint32_t)(m0 - row0 + 16 * i + rho);
      Q.old[i] = Q.res[i] = Q.y0[i] = Q.y1[i] = uint4{0, 0, 0, 0};
      Q.bits[i] = 0xffu;
      if constexpr (EP != 1 && (OPS & OP_OLD))
        Q.old[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yr, r * yb + 16 * g + nc * 2, 0, 0));
      if constexpr (EP != 0 && (OPS & OP_RES))
        Q.res[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(resr, r * rb + 16 * g, nc * 2, 0));
      if constexpr (EP == 2) {
        // ReLU bits: the chunk's 4 bytes of the row as one dword (the row's 4 lanes read the same word; byte g is this
        // lane's, extracted at use) — chunk pairs take both dwords with one 8-B load in prefetch() below
        if constexpr ((OPS & OP_MASK) != 0)
          if (!pairbits) Q.bits[i] = __builtin_amdgcn_raw_buffer_load_b32(mr, r * mrow, nc >> 3, 0);
        if constexpr (need_y0)
          Q.y0[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(y0r, r * nb + 16 * g, nc * 2, 0));
        if constexpr (dual)
          Q.y1[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(y1r, r * nb + 16 * g, nc * 2, 0));
      }
    }
  };
  // prefetch cursor (tile tp, iteration ip), restarted per tile
  int tp = 0, ip = 0;
  auto prefetch = [&](Pre<TM> (&Q)[CPI]) {
    const int m0 = mfirst + tp * tstride;
    pairbits = EP == 2 && (OPS & OP_MASK) != 0 && CPI == 2 && ip * CPI + 1 < nch;
#pragma unroll
    for (int cc = 0; cc < CPI; ++cc)
      if (ip * CPI + cc < nch) prefetch1(m0, ip * CPI + cc, Q[cc]);
    if constexpr (EP == 2 && (OPS & OP_MASK) != 0 && CPI == 2) {
      if (pairbits) {
        const int nc = nb0 + 32 * ip * CPI;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const uint32_t r = (uint32_t)(m0 - row0 + 16 * i + rho);
          const u32x2_t_ v = __builtin_bit_cast(u32x2_t_, __builtin_amdgcn_raw_buffer_load_b64(mr, r * mrow, nc >> 3, 0));
          Q[0].bits[i] = v[0];
          Q[CPI - 1].bits[i] = v[1];
        }
      }
    }
    if (++ip == nit) { ip = 0; ++tp; }
  };
  if (ntw > 0) load_a(mfirst);
  ev8_t a[TM][KS];
#pragma unroll 1
  for (int t = 0; t < ntw; ++t) {
    const int m0 = mfirst + t * tstride;
    // the tensor's last tile may run past its end: those rows' epilogue values are zeroed (their stores
    // are dropped by the buffer range, but a bias or input affine would leak into the statistics)
    const bool tail = m0 + MT > row_end;
    {
      // this tile's activations (lane: position m0 + 16 i + rho, k = 32 s + 8 g .. + 8), then the next
      // tile's raw loads
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          uint4 v = araw[i][s];
          const bool live = taps ? ((amask >> (i * KS + s)) & 1u) != 0 : xk[s] != OOB;
          if (AFF && live && !(tail && m0 + 16 * i + rho >= row_end)) {   // (padding stays zero)
            const int k0 = taps ? kc[s] : 32 * s + 8 * g;
            float f[8];
            unpack8(v, f);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float z = __builtin_fmaf(f[e], affs[k0 + e], affs[Ca + k0 + e]);
              f[e] = AFF == 2 ? fmaxf(z, 0.f) : z;
            }
            v = pack8_fast(f);
          }
          a[i][s] = __builtin_bit_cast(ev8_t, v);
        }
      if (t + 1 < ntw) load_a(m0 + tstride);
    }
    tp = t; ip = 0;
#pragma unroll
    for (int d = 0; d < PD - 1; ++d)
      if (d < nit) prefetch(P[d]);
#pragma unroll 1
    for (int it = 0; it < nit; ++it) {
      if (it + PD - 1 < nit) prefetch(P[PD - 1]);
      unsigned mbits[TM][CPI];   // EP 1: ReLU bytes of this iteration's chunks, stored together below
#pragma unroll
      for (int cc = 0; cc < CPI; ++cc) {
        const int c = it * CPI + cc;
        if (c >= nch) break;
        const int nl = 32 * c + 8 * g;   // this lane's 8 output channels (group-local)
        const int nc = nb0 + 32 * c;     // chunk's first channel
        // ---- MFMAs: D = W X^T, lane gets channels n..n+3 (half 0) and n+4..n+7 (half 1) of its position
        f32x4_t acc[TM][2];
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][0] = acc[i][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const char* wc = smem + (c * 2 * KS) * 1024 + lane * 16;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const ev8_t w0 = *reinterpret_cast<const ev8_t*>(wc + s * 1024);
          const ev8_t w1 = *reinterpret_cast<const ev8_t*>(wc + (KS + s) * 1024);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            acc[i][0] = PVA_MFMA16(w0, a[i][s], acc[i][0], 0, 0, 0);
            acc[i][1] = PVA_MFMA16(w1, a[i][s], acc[i][1], 0, 0, 0);
          }
        }
        // ---- epilogue (operands in P[0][cc])
        const Pre<TM>& E = P[0][cc];
        float cb[8], c2[8], c3[8], c4[8];   // per-channel constants of this lane's 8 channels (from LDS)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          cb[e] = cst[nl + e];
          c2[e] = EP == 1 ? cst[NG + nl + e] : 0.f;
          c3[e] = EP == 1 ? ((OPS & OP_RAFF) ? cst[2 * NG + nl + e] : 1.f) : (masky ? cst[NG + nl + e] : 0.f);
          c4[e] = EP == 1 ? ((OPS & OP_RAFF) ? cst[3 * NG + nl + e] : 0.f) : (masky ? cst[2 * NG + nl + e] : 0.f);
        }
        float s_a[8], s_b[8], s_c[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) { s_a[e] = 0.f; s_b[e] = 0.f; s_c[e] = 0.f; }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const uint32_t r = (uint32_t)(m0 - row0 + 16 * i + rho);
          const bool dead = tail && m0 + 16 * i + rho >= row_end;
          float v[8] = {acc[i][0][0], acc[i][0][1], acc[i][0][2], acc[i][0][3],
                        acc[i][1][0], acc[i][1][1], acc[i][1][2], acc[i][1][3]};
          if (EP == 1) {
            float rr[8];
            unpack8(E.res[i], rr);
            if constexpr ((OPS & OP_RAFF) != 0) {
#pragma unroll
              for (int e = 0; e < 8; ++e) rr[e] = __builtin_fmaf(rr[e], c3[e], c4[e]);
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaxf(__builtin_fmaf(v[e], cb[e], c2[e]) + rr[e], 0.f);
            const uint4 pk = pack8_fast(v);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, pk), yr, r * yb + 16 * g + nc * 2, 0,
                                                   ST_AUX);
            // bit = stored 16-bit value > 0 (res_out's convention)
            mbits[i][cc] = relu_bits8(pk);
          } else if (EP == 0) {
            float o[8];
            unpack8(E.old[i], o);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += cb[e] + o[e];
            if (tail && dead)
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] = 0.f;
            const uint4 pk = pack8_fast(v);
            if (!nostore)   // (statistics-only pass of a narrow BN fold: the output is never stored)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, pk), yr, r * yb + 16 * g + nc * 2, 0,
                                                     ST_AUX);
            if (do_stats) {
              float q[8];
              unpack8(pk, q);
#pragma unroll
              for (int e = 0; e < 8; ++e) { s_a[e] += q[e]; s_b[e] += q[e] * q[e]; }
            }
          } else {
            float o[8], rr[8], y0[8];
            unpack8(E.old[i], o);
            unpack8(E.res[i], rr);
            unpack8(E.y0[i], y0);
            unsigned bits = (OPS & OP_MASK) ? (E.bits[i] >> (8 * g)) & 0xffu : E.bits[i];
            if (masky) {
#pragma unroll
              for (int e = 0; e < 8; ++e)
                if (!(__builtin_fmaf(y0[e], c3[e], c4[e]) > 0.f)) bits &= ~(1u << e);
            }
            if (tail && dead) bits = 0;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              // bit e -> all-ones / zero (one signed bitfield extract), ANDed onto the float bits
              const unsigned keep = (unsigned)__builtin_amdgcn_sbfe((int)bits, e, 1);
              v[e] = __uint_as_float(__float_as_uint(v[e] + o[e] + rr[e] + cb[e]) & keep);
            }
            const uint4 pk = pack8_fast(v);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, pk), yr, r * yb + 16 * g + nc * 2, 0,
                                                   ST_AUX);
            if (do_stats) {
              float q[8], y1[8];
              unpack8(pk, q);
              unpack8(E.y1[i], y1);
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                s_a[e] += q[e];
                if (stat_b) s_b[e] += q[e] * y0[e];
                if (dual) s_c[e] += q[e] * y1[e];
              }
            }
          }
        }
        if (do_stats) {
          if constexpr (stat_b) {
            // lane rho ends with element rho of {s_a[8], s_b[8]} (stat rho >> 3, channel rho & 7)
            float t16[16];
#pragma unroll
            for (int e = 0; e < 8; ++e) { t16[e] = s_a[e]; t16[8 + e] = s_b[e]; }
            rs16<16>(t16, lane);
            sw[(rho >> 3) * NG + nl + (rho & 7)] += t16[0];
          } else {   // lanes 2e and 2e + 1 end with channel e
            rs16<8>(s_a, lane);
            if (!(rho & 1)) sw[nl + (rho >> 1)] += s_a[0];
          }
          if constexpr (dual) {   // third statistic
            rs16<8>(s_c, lane);
            if (!(rho & 1)) sw[2 * NG + nl + (rho >> 1)] += s_c[0];
          }
        }
      }
      if constexpr (EP == 1) {
        // a row's ReLU bytes of the iteration's chunks are contiguous (chunk c, lane group g -> byte 4c + g): gathered
        // from the row's 4 lanes (lane rho + 16 g) and written by lane g = 0 as one 4-B / 8-B store, instead of one
        // byte store per lane and chunk (measured ~8 % of the residual-output pass, tools/probe/fres_probe.py)
        const int c0 = it * CPI;
        const bool pair = CPI == 2 && c0 + 1 < nch;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          unsigned lo = mbits[i][0] << (8 * g), hi = CPI == 2 ? mbits[i][CPI - 1] << (8 * g) : 0u;
          lo |= __shfl_xor(lo, 16, 64);
          lo |= __shfl_xor(lo, 32, 64);
          if (CPI == 2) {
            hi |= __shfl_xor(hi, 16, 64);
            hi |= __shfl_xor(hi, 32, 64);
          }
          const uint32_t r = (uint32_t)(m0 - row0 + 16 * i + rho);
          const uint32_t mo = g == 0 ? r * mrow + ((nb0 + 32 * c0) >> 3) : 0x80000000u;   // other lanes: dropped
          if (pair)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t_, (uint2){lo, hi}), mor, mo, 0, 0);
          else
            __builtin_amdgcn_raw_buffer_store_b32(lo, mor, mo, 0, 0);
        }
      }
#pragma unroll
      for (int d = 0; d < PD - 1; ++d)
#pragma unroll
        for (int cc = 0; cc < CPI; ++cc) P[d][cc] = P[d + 1][cc];
    }
  }
  if (!do_stats) return;
  __syncthreads();
  for (int i = tid; i < NST * NG; i += (NW * 64)) {
    const int k = i / NG, nl = i - k * NG, n = nb0 + nl;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += st_lds[w * NST * NG + i];
    if (EP == 2 && k > 0) {   // sum v * xhat = rstd (sum v y - mean sum v)
      const float* mean = k == 1 ? p.emean0 : p.emean1;
      const float* rstd = k == 1 ? p.erstd0 : p.erstd1;
      const bool have = k == 1 ? p.ey0 != nullptr : p.ey1 != nullptr;
      float s0 = 0.f;   // sum v over the waves (the same fixed order as above)
#pragma unroll
      for (int w = 0; w < NW; ++w) s0 += st_lds[w * NST * NG + nl];
      v = have ? (v - mean[n] * s0) * rstd[n] : 0.f;
    }
    if (EP == 2) p.epart[((int64_t)rblk * 3 + k) * N + n] = v;
    else p.stats[((int64_t)rblk * 2 + k) * N + n] = v;
  }
}

template <int KS, int TM, int EP, int AFF, int OPS, int PD, bool TP, int NW>
void launch_one(const ConvParams& p, int rpb, int gch, size_t lds, hipStream_t st) {
  // non-temporal (streaming) output stores for the BN-folded residual output, whose 16-B rows are never
  // re-read while L2-resident (measured +8 % on the res2 shape, scripts/pw_probe.py); the other epilogues
  // measured 1-3 % slower with them.  TM is the tile height at one chunk per iteration: chunk pairs halve
  // it, keeping the registers of a ring stage.  One-chunk groups (N = 32) run the single-chunk variant at
  // KS = 1 (the fast pathway's layers) and the pair variant (half a pair idle) otherwise.
  const int ngrp = ((p.Ngemm >> 5) + gch - 1) / gch;
  const dim3 grid(((p.M + rpb - 1) / rpb) * ngrp), block(NW * 64);
  // 4-wave workgroups: one ring stage less (the third wave per SIMD hides the latency instead), which brings the
  // residual-output and two-stream epilogues under the 168 VGPRs of three waves per SIMD
  constexpr int PDW = (NW == 4 && PD > 2) ? PD - 1 : PD;
  if constexpr (KS == 1) {
    if (gch < 2) {
      hipLaunchKernelGGL((conv_pw_kernel<KS, TM, EP, AFF, EP == 1, OPS, PDW, 1, TP, NW>), grid, block, lds, st, p, rpb, gch);
      return;
    }
  }
  hipLaunchKernelGGL((conv_pw_kernel<KS, (TM > 1 ? TM / 2 : 1), EP, AFF, EP == 1, OPS, PDW, 2, TP, NW>), grid, block, lds,
                     st, p, rpb, gch);
}

template <int KS, int TM, int EP, int OPS, int PD, bool TP, int NW>
void launch_aff(const ConvParams& p, int rpb, int gch, size_t lds, hipStream_t st) {
  switch (EP == 2 ? 0 : p.affine) {
    case 0: launch_one<KS, TM, EP, 0, OPS, PD, TP, NW>(p, rpb, gch, lds, st); break;
    case 1: launch_one<KS, TM, EP, 1, OPS, PD, TP, NW>(p, rpb, gch, lds, st); break;
    default: launch_one<KS, TM, EP, 2, OPS, PD, TP, NW>(p, rpb, gch, lds, st); break;
  }
}

// backward-BN epilogue: tile rows and ring depth sized by the 16-B operand streams an instantiation
// carries (a lane holds TM * 16 B per stream per ring stage)
template <int KS, int OPS, bool TP, int NW>
void launch_ep2(const ConvParams& p, int rpb, int gch, size_t lds, hipStream_t st) {
  constexpr int nops = ((OPS >> 0) & 1) + ((OPS >> 1) & 1) + ((OPS >> 2) & 1) + ((OPS >> 3) & 1);
  constexpr int TM0 = nops <= 1 ? 4 : 2;
  constexpr int TM = KS <= 2 ? TM0 : KS == 4 ? 2 : TM0 / 2;
  constexpr int PD = nops <= 2 ? 3 : 2;
  launch_one<KS, TM, 2, 0, OPS, PD, TP, NW>(p, rpb, gch, lds, st);
}

// the operand-stream combinations the dgrad epilogues produce (models/fused.py): the BN path (ReLU from
// affine(y0), + accumulate), and the residual-unit path (residual and / or ReLU bits with up to two BN
// inputs, + accumulate)
constexpr int EP2_OPS[] = {
    OP_Y0 | OP_MSC, OP_Y0 | OP_MSC | OP_OLD,
    0, OP_OLD, OP_RES, OP_RES | OP_OLD,
    OP_MASK, OP_MASK | OP_OLD, OP_MASK | OP_RES, OP_MASK | OP_RES | OP_OLD,
    OP_MASK | OP_Y0, OP_MASK | OP_Y0 | OP_OLD, OP_MASK | OP_Y0 | OP_RES, OP_MASK | OP_Y0 | OP_RES | OP_OLD,
    OP_MASK | OP_Y1, OP_MASK | OP_Y1 | OP_OLD, OP_MASK | OP_Y1 | OP_RES, OP_MASK | OP_Y1 | OP_RES | OP_OLD,
    OP_MASK | OP_Y0 | OP_Y1, OP_MASK | OP_Y0 | OP_Y1 | OP_OLD, OP_MASK | OP_Y0 | OP_Y1 | OP_RES,
    OP_MASK | OP_Y0 | OP_Y1 | OP_RES | OP_OLD};
constexpr int N_EP2_OPS = sizeof(EP2_OPS) / sizeof(EP2_OPS[0]);

template <int KS, bool TP, int NW, int I = 0>
bool launch_ep2_ops(const ConvParams& p, int ops, int rpb, int gch, size_t lds, hipStream_t st) {
  if constexpr (I < N_EP2_OPS) {
    if (ops == EP2_OPS[I]) {
      launch_ep2<KS, EP2_OPS[I], TP, NW>(p, rpb, gch, lds, st);
      return true;
    }
    return launch_ep2_ops<KS, TP, NW, I + 1>(p, ops, rpb, gch, lds, st);
  } else {
    return false;
  }
}

// forward epilogues: 64-row tiles (32 at K > 128), 3-deep ring; false: no instantiation for `ops`.  TP: the
// temporal-tap loader (no residual-output epilogue: that one belongs to the 1x1 conv_c)
template <int KS, bool TP, int NW>
bool launch_ks_tp(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st) {
  constexpr int TMF = KS <= 4 ? 4 : 2;
  if (ep == 1) {
    if constexpr (TP) return false;
    else {
      if (ops & OP_RAFF) launch_aff<KS, TMF, 1, OP_RES | OP_RAFF, 3, false, NW>(p, rpb, gch, lds, st);
      else launch_aff<KS, TMF, 1, OP_RES, 3, false, NW>(p, rpb, gch, lds, st);
      return true;
    }
  }
  if (ep == 0) {
    if (ops & OP_OLD) launch_aff<KS, TMF, 0, OP_OLD, 3, TP, NW>(p, rpb, gch, lds, st);
    else launch_aff<KS, TMF, 0, 0, 3, TP, NW>(p, rpb, gch, lds, st);
    return true;
  }
  return launch_ep2_ops<KS, TP, NW>(p, ops, rpb, gch, lds, st);
}

template <int KS, int NW>
bool launch_ks(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st) {
  return p.nt > 1 ? launch_ks_tp<KS, true, NW>(p, ep, ops, rpb, gch, lds, st)
                  : launch_ks_tp<KS, false, NW>(p, ep, ops, rpb, gch, lds, st);
}

}  // namespace

PVA_NS_END  // namespace PVA_NS
