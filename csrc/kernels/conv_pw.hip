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
//     chunks ahead through a register ring, so several chunks of loads stay in flight per wave (with only
//     8 waves per CU, a single chunk in flight capped these layers at ~3.5 TB/s by Little's law);
//   * per-channel epilogue constants are staged in LDS once per workgroup;
//   * output channels are permuted inside each 32-channel chunk so a lane's two accumulator fragments hold
//     8 CONSECUTIVE channels of one position: 16-B stores, 16-B residual / BN-input loads, and one
//     ReLU-mask byte per lane (no cross-lane shuffles);
//   * per-channel statistics are reduced across the 16 lanes of a fragment column by a butterfly
//     reduce-scatter (15 shuffles for 16 values) and accumulated per workgroup with LDS float adds
//     (like the split-K weight gradients: not bitwise run-to-run deterministic, so deterministic mode
//     never selects this kernel), then written as one partial slab per workgroup.
// Epilogues (EP): 0 plain (+bias, +accumulate, +forward BN statistics), 1 the BN-folded residual-unit
// output (conv_igemm's fres), 2 the backward-BN epilogue of the dgrads (conv_igemm's EPI 1).
#include "common.h"
#include "conv_params.h"
#include <algorithm>

namespace {

constexpr int PW_WAVES = 8;
constexpr int PW_THREADS = PW_WAVES * 64;
constexpr int PW_LDS = 156 * 1024;     // LDS budget of a workgroup (weights, statistics, constants)

// Butterfly reduce-scatter over the 16 lanes sharing lane >> 4: v[L] in; lane rho ends up holding the
// 16-lane total of element rho (L = 16) or of element rho >> 1 (L = 8) in v[0].
template <int L>
__device__ __forceinline__ void rs16(float (&v)[L], int lane) {
  static_assert(L == 8 || L == 16, "16 or 8 values");
#pragma unroll
  for (int st = 0; st < (L == 16 ? 4 : 3); ++st) {
    const int m = 8 >> st;
    const int half = L >> (st + 1);
    // blend through a bit mask: a plain ?: lets the compiler turn the select into a lane-dependent array
    // index, lowered as compare/select chains over the whole array (measured: ~500 extra instructions)
    const unsigned hm = (lane & m) ? 0xffffffffu : 0u;
#pragma unroll
    for (int j = 0; j < half; ++j) {
      const unsigned lo = __float_as_uint(v[j]), hi = __float_as_uint(v[j + half]);
      const unsigned x = (lo ^ hi) & hm;
      const float send = __uint_as_float(hi ^ x);   // up: lo, else hi
      const float keep = __uint_as_float(lo ^ x);   // up: hi, else lo
      v[j] = keep + __shfl_xor(send, m, 64);
    }
  }
  if (L == 8) v[0] += __shfl_xor(v[0], 1, 64);
}

// 16-B output store; NT: non-temporal (streaming) store hint
template <bool NT>
__device__ __forceinline__ void st16(uint16_t* dst, const uint4& v) {
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
  if constexpr (NT) __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_t*>(dst));
  else *reinterpret_cast<uint4*>(dst) = v;
}

// epilogue operands of one 32-channel chunk (members an epilogue does not use are optimised away)
template <int TM>
struct Pre {
  uint4 old[TM], res[TM], y0[TM], y1[TM];
  unsigned bits[TM];
};

template <int KS, int TM, int EP, int AFF, bool NTS>
__global__ __launch_bounds__(PW_THREADS) void conv_pw_kernel(const ConvParams p, int rpb, int gch) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NST = EP == 2 ? 3 : 2;
  constexpr int MT = 16 * TM;
  constexpr int PD = EP == 2 ? 2 : 3;   // prefetch ring depth (chunks)
  const int N = p.Ngemm, K = p.Cg;
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
  float* st_lds = reinterpret_cast<float*>(smem + wimg);   // [NST][NG] workgroup statistics
  float* cst = st_lds + NST * NG;                           // [4][NG] per-channel epilogue constants
  float* affs = cst + 4 * NG;                               // [2][K] input affine
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rho = lane & 15, g = lane >> 4;

  // ---- weight image: fragment f = (c * 2 + h) * KS + s, lane l's 16 B at f * 1024 + 16 l:
  //      row rho of half h of chunk c = output channel 32c + 8(rho >> 2) + 4h + (rho & 3), k = 32s + 8(l >> 4)
  const int units = nch * 2 * KS * 64;
  for (int u = tid; u < units; u += PW_THREADS) {
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
  if (do_stats)
    for (int i = tid; i < NST * NG; i += PW_THREADS) st_lds[i] = 0.f;
  if (AFF)
    for (int i = tid; i < K; i += PW_THREADS) { affs[i] = p.in_scale[i]; affs[K + i] = p.in_shift[i]; }
  // EP 1: fsc fsh rsc rsh ; EP 0 / 2: bias (0 when absent), mask-affine scale and shift
  for (int i = tid; i < NG; i += PW_THREADS) {
    const int n = nb0 + i;
    if (EP == 1) {
      cst[i] = p.fsc[n]; cst[NG + i] = p.fsh[n];
      cst[2 * NG + i] = p.rsc ? p.rsc[n] : 1.f; cst[3 * NG + i] = p.rsh ? p.rsh[n] : 0.f;
    } else {
      cst[i] = p.ebias ? p.ebias[n] : 0.f;
      if (EP == 2 && p.emsc) { cst[NG + i] = p.emsc[n]; cst[2 * NG + i] = p.emsh[n]; }
    }
  }
  __syncthreads();

  const int row0 = rblk * rpb;
  const int row_end = min(p.M, row0 + rpb);
  const int mrow = N >> 3;   // mask bytes per row
  const bool dual = EP == 2 && p.ey1 != nullptr;
  const bool masky = EP == 2 && p.emsc != nullptr;
  const bool need_y0 = EP == 2 && p.ey0 != nullptr && (masky || do_stats);

#pragma unroll 1
  for (int m0 = row0 + wid * MT; m0 < row_end; m0 += PW_WAVES * MT) {
    // ---- this tile's activations, once: lane holds position m0 + 16 i + rho, k = 32 s + 8 g .. + 8
    bf16x8_t a[TM][KS];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + 16 * i + rho;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int k0 = 32 * s + 8 * g;
        uint4 v = uint4{0, 0, 0, 0};
        if (m < row_end && k0 < K) {
          v = *reinterpret_cast<const uint4*>(p.x + (int64_t)m * p.ldx + k0);
          if (AFF) {
            float f[8];
            unpack8(v, f);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float z = __builtin_fmaf(f[e], affs[k0 + e], affs[K + k0 + e]);
              f[e] = AFF == 2 ? fmaxf(z, 0.f) : z;
            }
            v = pack8_fast(f);
          }
        }
        a[i][s] = __builtin_bit_cast(bf16x8_t, v);
      }
    }
    // epilogue operands of chunk c are issued PD - 1 chunks ahead (a register ring), so PD - 1 chunks of
    // loads stay in flight behind the MFMAs and stores of the current one
    Pre<TM> P[PD];
    auto prefetch = [&](int c, Pre<TM>& Q) {
      const int n = nb0 + 32 * c + 8 * g;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + 16 * i + rho;
        Q.old[i] = Q.res[i] = Q.y0[i] = Q.y1[i] = uint4{0, 0, 0, 0};
        Q.bits[i] = 0xffu;
        if (m >= row_end) continue;
        if (EP != 1 && p.accum) Q.old[i] = *reinterpret_cast<const uint4*>(p.y + (int64_t)m * p.ldy + n);
        if (EP != 0 && p.eres) Q.res[i] = *reinterpret_cast<const uint4*>(p.eres + (int64_t)m * p.ldr + n);
        if (EP == 2) {
          if (p.emask) Q.bits[i] = p.emask[(int64_t)m * mrow + (n >> 3)];
          if (need_y0) Q.y0[i] = *reinterpret_cast<const uint4*>(p.ey0 + (int64_t)m * N + n);
          if (dual && do_stats) Q.y1[i] = *reinterpret_cast<const uint4*>(p.ey1 + (int64_t)m * N + n);
        }
      }
    };
#pragma unroll
    for (int d = 0; d < PD - 1; ++d)
      if (d < nch) prefetch(d, P[d]);
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      const int nl = 32 * c + 8 * g;   // this lane's 8 output channels (group-local)
      const int n = nb0 + nl;
      if (c + PD - 1 < nch) prefetch(c + PD - 1, P[PD - 1]);
      // ---- MFMAs: D = W X^T, lane gets channels n..n+3 (half 0) and n+4..n+7 (half 1) of its position
      f32x4_t acc[TM][2];
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[i][0] = acc[i][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const char* wc = smem + (c * 2 * KS) * 1024 + lane * 16;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const bf16x8_t w0 = *reinterpret_cast<const bf16x8_t*>(wc + s * 1024);
        const bf16x8_t w1 = *reinterpret_cast<const bf16x8_t*>(wc + (KS + s) * 1024);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, a[i][s], acc[i][0], 0, 0, 0);
          acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, a[i][s], acc[i][1], 0, 0, 0);
        }
      }
      // ---- epilogue (operands in P[0])
      const uint4* e_old = P[0].old;
      const uint4* e_res = P[0].res;
      const uint4* e_y0 = P[0].y0;
      const uint4* e_y1 = P[0].y1;
      const unsigned* e_bits = P[0].bits;
      float cb[8], c2[8], c3[8], c4[8];   // per-channel constants of this lane's 8 channels (from LDS)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        cb[e] = cst[nl + e];
        c2[e] = EP == 1 ? cst[NG + nl + e] : 0.f;
        c3[e] = EP == 1 ? cst[2 * NG + nl + e] : (masky ? cst[NG + nl + e] : 0.f);
        c4[e] = EP == 1 ? cst[3 * NG + nl + e] : (masky ? cst[2 * NG + nl + e] : 0.f);
      }
      float s_a[8], s_b[8], s_c[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { s_a[e] = 0.f; s_b[e] = 0.f; s_c[e] = 0.f; }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + 16 * i + rho;
        if (m >= row_end) continue;
        float v[8] = {acc[i][0][0], acc[i][0][1], acc[i][0][2], acc[i][0][3],
                      acc[i][1][0], acc[i][1][1], acc[i][1][2], acc[i][1][3]};
        if (EP == 1) {
          float r[8];
          unpack8(e_res[i], r);
#pragma unroll
          for (int e = 0; e < 8; ++e) r[e] = __builtin_fmaf(r[e], c3[e], c4[e]);   // identity: 1, 0
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(__builtin_fmaf(v[e], cb[e], c2[e]) + r[e], 0.f);
          const uint4 pk = pack8_fast(v);
          st16<NTS>(p.y + (int64_t)m * p.ldy + n, pk);
          const uint32_t w4[4] = {pk.x, pk.y, pk.z, pk.w};
          unsigned bits = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {   // bit = stored bf16 > 0 (res_out's convention)
            bits |= ((w4[e] & 0x7fffu) != 0 && !(w4[e] & 0x8000u)) ? 1u << (2 * e) : 0u;
            bits |= ((w4[e] & 0x7fff0000u) != 0 && !(w4[e] & 0x80000000u)) ? 1u << (2 * e + 1) : 0u;
          }
          p.emask_out[(int64_t)m * mrow + (n >> 3)] = (uint8_t)bits;
        } else if (EP == 0) {
          float o[8];
          unpack8(e_old[i], o);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += cb[e] + o[e];
          const uint4 pk = pack8_fast(v);
          st16<NTS>(p.y + (int64_t)m * p.ldy + n, pk);
          if (do_stats) {
            float q[8];
            unpack8(pk, q);
#pragma unroll
            for (int e = 0; e < 8; ++e) { s_a[e] += q[e]; s_b[e] += q[e] * q[e]; }
          }
        } else {
          float o[8], r[8], y0[8];
          unpack8(e_old[i], o);
          unpack8(e_res[i], r);
          unpack8(e_y0[i], y0);
          unsigned bits = e_bits[i];
          if (masky) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (!(__builtin_fmaf(y0[e], c3[e], c4[e]) > 0.f)) bits &= ~(1u << e);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float t = v[e] + o[e] + r[e] + cb[e];
            v[e] = (bits >> e) & 1u ? t : 0.f;
          }
          const uint4 pk = pack8_fast(v);
          st16<NTS>(p.y + (int64_t)m * p.ldy + n, pk);
          if (do_stats) {
            float q[8], y1[8];
            unpack8(pk, q);
            unpack8(e_y1[i], y1);
#pragma unroll
            for (int e = 0; e < 8; ++e) { s_a[e] += q[e]; s_b[e] += q[e] * y0[e]; s_c[e] += q[e] * y1[e]; }
          }
        }
      }
      if (do_stats) {
        // lane rho ends with element rho of {s_a[8], s_b[8]} (stat rho >> 3, channel rho & 7)
        float t[16];
#pragma unroll
        for (int e = 0; e < 8; ++e) { t[e] = s_a[e]; t[8 + e] = s_b[e]; }
        rs16<16>(t, lane);
        atomicAdd(st_lds + (rho >> 3) * NG + nl + (rho & 7), t[0]);
        if (EP == 2 && dual) {   // third statistic: lanes 2e and 2e + 1 end with channel e
          rs16<8>(s_c, lane);
          if (!(rho & 1)) atomicAdd(st_lds + 2 * NG + nl + (rho >> 1), s_c[0]);
        }
      }
#pragma unroll
      for (int d = 0; d < PD - 1; ++d) P[d] = P[d + 1];
    }
  }
  if (!do_stats) return;
  __syncthreads();
  for (int i = tid; i < NST * NG; i += PW_THREADS) {
    const int k = i / NG, nl = i - k * NG, n = nb0 + nl;
    float v = st_lds[i];
    if (EP == 2 && k > 0) {   // sum v * xhat = rstd (sum v y - mean sum v)
      const float* mean = k == 1 ? p.emean0 : p.emean1;
      const float* rstd = k == 1 ? p.erstd0 : p.erstd1;
      const bool have = k == 1 ? p.ey0 != nullptr : p.ey1 != nullptr;
      v = have ? (v - mean[n] * st_lds[nl]) * rstd[n] : 0.f;
    }
    if (EP == 2) p.epart[((int64_t)rblk * 3 + k) * N + n] = v;
    else p.stats[((int64_t)rblk * 2 + k) * N + n] = v;
  }
}

template <int KS, int TM, int EP, bool NTS>
void launch_ep_nt(const ConvParams& p, int rpb, int gch, size_t lds, hipStream_t st) {
  const int ngrp = ((p.Ngemm >> 5) + gch - 1) / gch;
  const dim3 grid(((p.M + rpb - 1) / rpb) * ngrp), block(PW_THREADS);
  if constexpr (EP == 2) {
    hipLaunchKernelGGL((conv_pw_kernel<KS, TM, 2, 0, NTS>), grid, block, lds, st, p, rpb, gch);
  } else {
    switch (p.affine) {
      case 0: hipLaunchKernelGGL((conv_pw_kernel<KS, TM, EP, 0, NTS>), grid, block, lds, st, p, rpb, gch); break;
      case 1: hipLaunchKernelGGL((conv_pw_kernel<KS, TM, EP, 1, NTS>), grid, block, lds, st, p, rpb, gch); break;
      default: hipLaunchKernelGGL((conv_pw_kernel<KS, TM, EP, 2, NTS>), grid, block, lds, st, p, rpb, gch); break;
    }
  }
}

// non-temporal (streaming) output stores for the BN-folded residual output, whose 16-B rows are never
// re-read while L2-resident (measured +8 % on the res2 shape, scripts/pw_probe.py); the other epilogues
// measured 1-3 % slower with them
template <int KS, int TM, int EP>
void launch_ep(const ConvParams& p, int rpb, int gch, size_t lds, hipStream_t st) {
  launch_ep_nt<KS, TM, EP, EP == 1>(p, rpb, gch, lds, st);
}

// forward epilogues: 64-row tiles (32 at K > 128); the backward-BN epilogue carries 4 operand rows per
// position through a 2-deep ring: 32-row tiles (16 at K > 128) keep it in registers
template <int KS>
void launch_ks(const ConvParams& p, int ep, int rpb, int gch, size_t lds, hipStream_t st) {
  constexpr int TMF = KS <= 4 ? 4 : 2;
  if (ep == 2) launch_ep<KS, (KS <= 4 ? 2 : 1), 2>(p, rpb, gch, lds, st);
  else if (ep == 1) launch_ep<KS, TMF, 1>(p, rpb, gch, lds, st);
  else launch_ep<KS, TMF, 0>(p, rpb, gch, lds, st);
}

inline int pw_ks(int K) {
  const int s = (K + 31) / 32;
  return s <= 1 ? 1 : s <= 2 ? 2 : s <= 4 ? 4 : 8;
}

}  // namespace

// rows per workgroup of a pointwise launch configuration (cfg bits 0-1)
int conv_pw_rows(int cfg) { return 1024 << (cfg & 3); }

// 1 when the geometry is a dense 1x1x1 unit-stride unpadded GEMM the pointwise kernel can run
int conv_pw_legal(const ConvParams& p, int chunk) {
  if (chunk != 8) return 0;
  if (p.nt != 1 || p.nh != 1 || p.nw != 1 || p.check) return 0;
  if (p.ast != 1 || p.ash != 1 || p.asw != 1 || p.aot != 0 || p.aoh != 0 || p.aow != 0) return 0;
  if (p.Gt != p.Rt || p.Gh != p.Rh || p.Gw != p.Rw) return 0;
  if (p.ost != 1 || p.osh != 1 || p.osw != 1 || p.ort != 0 || p.orh != 0 || p.orw != 0) return 0;
  if (p.Ot != p.Rt || p.Oh != p.Rh || p.Ow != p.Rw) return 0;
  if (p.Kfull != p.Cg || p.Cg % 8 != 0 || p.Cg > 256 || p.Ngemm % 32 != 0) return 0;
  if (p.ldx % 8 != 0 || p.ldy % 8 != 0) return 0;
  return 1;
}

// 32-channel chunks per output-channel group: the largest group whose weight image, statistics and epilogue
// constants fit the LDS budget, then balanced over the groups (equal work per workgroup)
static int pw_group_chunks(int N, int ks, int nst, int aff_bytes) {
  const int nch = N / 32;
  const int per_chunk = 2 * ks * 1024 + (nst + 4) * 32 * 4;
  const int gmax = std::max(1, (PW_LDS - aff_bytes) / per_chunk);
  const int ngrp = (nch + gmax - 1) / gmax;
  return (nch + ngrp - 1) / ngrp;
}

void conv_pw_launch(const ConvParams& p, int cfg, hipStream_t st) {
  const bool ep2 = !p.fres && (p.eres || p.emask || p.epart);
  const int ep = p.fres ? 1 : (ep2 ? 2 : 0);
  const int ks = pw_ks(p.Cg);
  const int nst = ep == 2 ? 3 : 2;
  const int aff_bytes = p.affine ? 2 * p.Cg * 4 : 0;
  const int gch = pw_group_chunks(p.Ngemm, ks, nst, aff_bytes);
  const int NG = gch * 32;
  const size_t lds = (size_t)gch * 2 * ks * 1024 + (size_t)(nst + 4) * NG * 4 + aff_bytes;
  const int rpb = conv_pw_rows(cfg);
  switch (ks) {
    case 1: launch_ks<1>(p, ep, rpb, gch, lds, st); break;
    case 2: launch_ks<2>(p, ep, rpb, gch, lds, st); break;
    case 4: launch_ks<4>(p, ep, rpb, gch, lds, st); break;
    default: launch_ks<8>(p, ep, rpb, gch, lds, st); break;
  }
}
