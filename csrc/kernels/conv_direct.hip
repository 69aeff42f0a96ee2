// Direct-to-register implicit-GEMM 3-D convolution for NARROW convs (Ngemm <= 64): the fast pathway of
// SlowFast (8-64 channels), the lateral fusions and narrow dgrads.
//
// Why a second conv kernel: with N <= 64 one wave covers every output channel, so nothing is gained by
// staging the gathered activations through LDS for re-use across waves.  In NDHWC the MFMA operand of
// one lane — 8 consecutive k = 8 channels of one tap of one output position — is ONE contiguous 16-B
// chunk in memory, so every lane loads its own fragment straight from global memory into VGPRs
// (raw buffer loads; padding taps use an out-of-range offset and the buffer unit returns zeros).  No LDS
// round trip and no barrier in the main loop; only the (tiny) packed weights live in LDS, staged once
// per workgroup, read as conflict-free ds_read_b128 fragments (row pitch = 16 B x odd).
//
//   * 4 waves per workgroup; each wave walks RT x 16 output rows at a time through a row range of
//     `rows_per_block` rows; per k-step (32 = 4 chunks of 8 channels) a lane issues RT 16-B loads,
//     NB ds_read_b128 and RT x NB MFMA 16x16x32 (operands swapped: D = W * X^T, so each lane ends up
//     with 4 consecutive channels of one position -> 8-B stores, like conv_igemm.hip).
//   * The chunk -> (tap offset, channel offset, tap coordinates) table is built once per workgroup in
//     LDS, so the k-loop does no integer division.
//   * Consumer-side BN(+ReLU) of the producer is applied to the fragment in registers (valid taps only:
//     padding stays zero, as in the reference where the conv pads the normalised activation).
//   * Epilogues are those of conv_igemm.hip, computed straight from the fragment: EPI 0 = store (+old
//     value when accumulating) + forward BN partial sums of the bf16-rounded output; EPI 1 = the dgrad
//     backward-BN epilogue (+residual, ReLU-bit / own-affine mask, partial sums of v, v*xhat0, v*xhat1).
//     Partial sums are per workgroup (tile = workgroup), reduced in a fixed order: deterministic.
#include "common.h"
#include "conv_params.h"

PVA_NS_BEGIN

namespace {

constexpr int DNT = 256;          // threads per workgroup (4 waves)
constexpr unsigned DOOB = 0xFFFFFFF0u;

// Division by a launch-constant divisor d >= 1 of n < 2^31 (round-up multiplier, Granlund-Montgomery):
// q = (umulhi(n, m) + n) >> s.  The row decomposition of every row group costs 3 of these instead of
// 3 integer divisions (~40 VALU ops each).
struct FastDiv {
  uint32_t m, s, d;
};

inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  const uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  return FastDiv{(uint32_t)m, s, d};
}

__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return (int)((__umulhi((uint32_t)n, f.m) + (uint32_t)n) >> f.s);
}

// NB: 16-channel output blocks (N <= 16*NB); RT: 16-row groups per wave iteration; KB: k-steps whose loads
// are in flight together
template <int NB, int EPI, int RT, int KB>
__global__ __launch_bounds__(DNT) void conv_direct_kernel(const ConvParams p, int rows_per_block, int KS,
                                                          FastDiv dTHW, FastDiv dHW, FastDiv dW) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int frow = lane & 15, fq = lane >> 4;
  const int taps = p.nt * p.nh * p.nw;
  const int cpt = p.Cg >> 3;                 // chunks per tap
  const int nchunks = taps * cpt;
  const int NCH = KS * 4;                    // chunks incl. zero padding to a whole k-step
  const int pitch = KS * 32 + 8;             // weight row pitch (bf16): 16 B x odd -> conflict-free

  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* wl = reinterpret_cast<uint16_t*>(smem);                           // [NB*16][pitch]
  int4* tab = reinterpret_cast<int4*>(smem + NB * 16 * pitch * 2);            // [NCH]
  float* aff = reinterpret_cast<float*>(tab + NCH);                           // [2][Cg]
  float* red = aff + (p.affine ? 2 * p.Cg : 0);                               // [4][3][NB*16]
  float* mk = red + 4 * 3 * NB * 16;                                          // [2][NB*16] own-affine mask

  // ---- stage the packed weights (rows >= N and chunks >= nchunks are zero) and the chunk table ----
  for (int i = tid; i < NB * 16 * NCH; i += DNT) {
    const int n = i / NCH, c = i - n * NCH;
    uint4 v = uint4{0, 0, 0, 0};
    if (n < p.Ngemm && c < nchunks) {
      const int tap = c / cpt, cin0 = (c - tap * cpt) << 3;
      const int jw = tap % p.nw, jh = (tap / p.nw) % p.nh, jt = tap / (p.nw * p.nh);
      const int tw = ((p.bt0 + jt * p.bts) * p.kh + (p.bh0 + jh * p.bhs)) * p.kw + (p.bw0 + jw * p.bws);
      v = *reinterpret_cast<const uint4*>(p.w + (int64_t)n * p.Kfull + tw * p.Cg + cin0);
    }
    *reinterpret_cast<uint4*>(wl + n * pitch + c * 8) = v;
  }
  for (int c = tid; c < NCH; c += DNT) {
    int4 e;
    if (c < nchunks) {
      const int tap = c / cpt, cin0 = (c - tap * cpt) << 3;
      const int jw = tap % p.nw, jh = (tap / p.nw) % p.nh, jt = tap / (p.nw * p.nh);
      e.x = p.dir * ((jt * p.Gh + jh) * p.Gw + jw) * p.ldx + cin0;
      e.y = p.dir * jt; e.z = p.dir * jh; e.w = (p.dir * jw) * 65536 + cin0;   // dw in the high half
    } else {
      e.x = 0; e.y = 1 << 24; e.z = 0; e.w = 0;   // padding chunk: the t test always fails -> zeros
    }
    tab[c] = e;
  }
  if (p.affine)
    for (int i = tid; i < p.Cg; i += DNT) { aff[i] = p.in_scale[i]; aff[p.Cg + i] = p.in_shift[i]; }
  if (EPI == 1 && p.emsc != nullptr && p.epart != nullptr)
    for (int i = tid; i < NB * 16; i += DNT) {
      mk[i] = i < p.Ngemm ? p.emsc[i] : 0.f;
      mk[NB * 16 + i] = i < p.Ngemm ? p.emsh[i] : 0.f;
    }
  __syncthreads();

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.xbytes, 0x00020000);
  const int RHW = p.Rh * p.Rw, RTHW = p.Rt * RHW;
  const int GHW = p.Gh * p.Gw, GTHW = p.Gt * GHW;
  const bool dense_rows = p.ost == 1 && p.osh == 1 && p.osw == 1 && p.Rt == p.Ot && p.Rh == p.Oh && p.Rw == p.Ow;
  const bool do_stats = EPI == 0 && p.stats != nullptr;
  const bool do_bstats = EPI == 1 && p.epart != nullptr;
  const bool dual = EPI == 1 && p.ey1 != nullptr;
  const bool masky = do_bstats && p.emsc != nullptr;

  float acc1[NB][4], acc2[NB][4], acc3[NB][4];   // EPI0: sum, sumsq ; EPI1: sum v, sum v*y0, sum v*y1
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      acc1[nb][r] = 0.f; acc2[nb][r] = 0.f; acc3[nb][r] = 0.f;
    }

  const int rbeg = blockIdx.x * rows_per_block;
  const int rend = min(p.M, rbeg + rows_per_block);
  const char* wfrag = reinterpret_cast<const char*>(wl) + frow * pitch * 2 + fq * 16;

  for (int base = rbeg + wid * RT * 16; base < rend; base += 4 * RT * 16) {
    int roff[RT], rt_[RT], rh_[RT], rw_[RT], pos[RT];
    bool rok[RT];
#pragma unroll
    for (int g = 0; g < RT; ++g) {
      const int m = base + g * 16 + frow;
      rok[g] = m < rend;
      const int mm = rok[g] ? m : rbeg;
      const int b = fdiv(mm, dTHW);
      int r = mm - b * RTHW;
      const int qt = fdiv(r, dHW); r -= qt * RHW;
      const int qh = fdiv(r, dW); const int qw = r - qh * p.Rw;
      rt_[g] = qt * p.ast + p.aot; rh_[g] = qh * p.ash + p.aoh; rw_[g] = qw * p.asw + p.aow;
      roff[g] = (b * GTHW + (rt_[g] * p.Gh + rh_[g]) * p.Gw + rw_[g]) * p.ldx;
      pos[g] = dense_rows ? mm
                          : ((b * p.Ot + qt * p.ost + p.ort) * p.Oh + qh * p.osh + p.orh) * p.Ow + qw * p.osw + p.orw;
    }
    f32x4_t acc[RT][NB];
#pragma unroll
    for (int g = 0; g < RT; ++g)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[g][nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // KB k-steps of loads are issued together (RT x KB 16-B loads in flight per lane) before any of them
    // is consumed: the loop is latency-bound, not MFMA- or bandwidth-bound
    for (int s0 = 0; s0 < KS; s0 += KB) {
      uint4 a[KB][RT];
      unsigned okm = 0;
      int cin0[KB];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int s = s0 + kb;
        const int4 e = tab[min(s, KS - 1) * 4 + fq];
        const int dw = e.w >> 16;
        cin0[kb] = e.w & 0xffff;
#pragma unroll
        for (int g = 0; g < RT; ++g) {
          const bool ok = s < KS && rok[g] && (unsigned)(rt_[g] + e.y) < (unsigned)p.Gt &&
                          (unsigned)(rh_[g] + e.z) < (unsigned)p.Gh && (unsigned)(rw_[g] + dw) < (unsigned)p.Gw;
          okm |= (unsigned)ok << (kb * RT + g);
          a[kb][g] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   xr, ok ? (roff[g] + e.x) * 2 : (int)DOOB, 0, 0));
        }
      }
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int s = s0 + kb;
        if (s >= KS) break;   // wave-uniform
        ev8_t bw[NB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          bw[nb] = *reinterpret_cast<const ev8_t*>(wfrag + nb * 16 * pitch * 2 + s * 64);
        if (p.affine) {
          const float* sp = aff + cin0[kb];
          const f32x4_t c0 = *reinterpret_cast<const f32x4_t*>(sp);
          const f32x4_t c1 = *reinterpret_cast<const f32x4_t*>(sp + 4);
          const f32x4_t h0 = *reinterpret_cast<const f32x4_t*>(sp + p.Cg);
          const f32x4_t h1 = *reinterpret_cast<const f32x4_t*>(sp + p.Cg + 4);
          const float sc8[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
          const float sh8[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
#pragma unroll
          for (int g = 0; g < RT; ++g) {
            float f[8];
            unpack8(a[kb][g], f);
#pragma unroll
            for (int k = 0; k < 8; ++k) f[k] = __builtin_fmaf(f[k], sc8[k], sh8[k]);
            uint4 v = pack8_fast(f);
            if (p.affine == 2) v = relu_e16x8(v);
            a[kb][g] = (okm >> (kb * RT + g)) & 1u ? v : uint4{0, 0, 0, 0};
          }
        }
#pragma unroll
        for (int g = 0; g < RT; ++g) {
          const ev8_t av = __builtin_bit_cast(ev8_t, a[kb][g]);
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[g][nb] = PVA_MFMA16(bw[nb], av, acc[g][nb], 0, 0, 0);
        }
      }
    }

    // ---- epilogue straight from the fragments: lane = position (frow), channels n = nb*16+4*fq+r ----
#pragma unroll
    for (int g = 0; g < RT; ++g) {
      if (!rok[g]) continue;
      const int ps = pos[g];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int n = nb * 16 + 4 * fq;
        if (n >= p.Ngemm) continue;
        float v[4] = {acc[g][nb][0], acc[g][nb][1], acc[g][nb][2], acc[g][nb][3]};
        uint16_t* dst = p.y + (int64_t)ps * p.ldy + n;
        if (p.accum) {
          float o[4];
          unpack4(*reinterpret_cast<const uint2*>(dst), o);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += o[r];
        }
        if constexpr (EPI == 1) {
          if (p.eres) {
            float o[4];
            unpack4(*reinterpret_cast<const uint2*>(p.eres + (int64_t)ps * p.ldr + n), o);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += o[r];
          }
          unsigned bits = 0xfu;
          if (p.emask) bits = (p.emask[(int64_t)ps * (p.Ngemm >> 3) + (n >> 3)] >> (n & 7)) & 0xfu;
          float y0[4] = {0.f, 0.f, 0.f, 0.f}, y1[4] = {0.f, 0.f, 0.f, 0.f};
          if (do_bstats) {
            if (p.ey0) unpack4(*reinterpret_cast<const uint2*>(p.ey0 + (int64_t)ps * p.Ngemm + n), y0);
            if (dual) unpack4(*reinterpret_cast<const uint2*>(p.ey1 + (int64_t)ps * p.Ngemm + n), y1);
            if (masky) {
              const f32x4_t ms = *reinterpret_cast<const f32x4_t*>(mk + n);
              const f32x4_t mh = *reinterpret_cast<const f32x4_t*>(mk + NB * 16 + n);
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (!(y0[r] * ms[r] + mh[r] > 0.f)) bits &= ~(1u << r);
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bits >> r) & 1u ? v[r] : 0.f;
          const uint2 pk = pack4(v);
          *reinterpret_cast<uint2*>(dst) = pk;
          if (do_bstats) {
            float q[4];
            unpack4(pk, q);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              acc1[nb][r] += q[r];
              acc2[nb][r] += q[r] * y0[r];
              acc3[nb][r] += q[r] * y1[r];
            }
          }
        } else {
          const uint2 pk = pack4(v);
          *reinterpret_cast<uint2*>(dst) = pk;
          if (do_stats) {
            float q[4];
            unpack4(pk, q);
#pragma unroll
            for (int r = 0; r < 4; ++r) { acc1[nb][r] += q[r]; acc2[nb][r] += q[r] * q[r]; }
          }
        }
      }
    }
  }

  // ---- per-workgroup partial sums: 16-lane reduce, one LDS slot per wave, fixed-order sum ----
  if (!(do_stats || do_bstats)) return;
  constexpr int NBW = NB * 16;
  const int nq = EPI == 1 ? 3 : 2;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a1 = sum16(acc1[nb][r]), a2 = sum16(acc2[nb][r]), a3 = EPI == 1 ? sum16(acc3[nb][r]) : 0.f;
      if (frow == 0) {
        const int nl = nb * 16 + 4 * fq + r;
        red[(wid * 3 + 0) * NBW + nl] = a1;
        red[(wid * 3 + 1) * NBW + nl] = a2;
        red[(wid * 3 + 2) * NBW + nl] = a3;
      }
    }
  __syncthreads();
  for (int i = tid; i < NBW; i += DNT) {
    if (i >= p.Ngemm) continue;
    float t[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      t[k] = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) t[k] += red[(w * 3 + k) * NBW + i];
    }
    if (EPI == 1) {
      // no y0 (BN-folded conv_c: its raw output does not exist): only the sums of v and v*xhat1
      const float m0 = p.ey0 ? p.emean0[i] : 0.f, r0 = p.ey0 ? p.erstd0[i] : 0.f;
      t[1] = (t[1] - m0 * t[0]) * r0;
      t[2] = dual ? (t[2] - p.emean1[i] * t[0]) * p.erstd1[i] : 0.f;
      for (int k = 0; k < nq; ++k) p.epart[((int64_t)blockIdx.x * 3 + k) * p.Ngemm + i] = t[k];
    } else {
      p.stats[((int64_t)blockIdx.x * 2) * p.Ngemm + i] = t[0];
      p.stats[((int64_t)blockIdx.x * 2 + 1) * p.Ngemm + i] = t[1];
    }
  }
}

inline int direct_ks(const ConvParams& p) { return (p.nt * p.nh * p.nw * (p.Cg >> 3) + 3) / 4; }

inline size_t direct_lds(const ConvParams& p, int NB) {
  const int KS = direct_ks(p);
  return (size_t)NB * 16 * (KS * 32 + 8) * 2 + KS * 4 * 16 + (p.affine ? 2 * p.Cg * 4 : 0) + (4 * 3 + 2) * NB * 16 * 4;
}

template <int NB, int RT, int KB>
void direct_launch_cfg(const ConvParams& p, int rpb, bool epi, hipStream_t s) {
  const int KS = direct_ks(p);
  const dim3 grid((p.M + rpb - 1) / rpb), block(DNT);
  const size_t lds = direct_lds(p, NB);
  const FastDiv a = make_fastdiv((uint32_t)(p.Rt * p.Rh * p.Rw)), b = make_fastdiv((uint32_t)(p.Rh * p.Rw)),
                c = make_fastdiv((uint32_t)p.Rw);
  if (epi) hipLaunchKernelGGL((conv_direct_kernel<NB, 1, RT, KB>), grid, block, lds, s, p, rpb, KS, a, b, c);
  else hipLaunchKernelGGL((conv_direct_kernel<NB, 0, RT, KB>), grid, block, lds, s, p, rpb, KS, a, b, c);
}

// loads in flight per lane = RT x KB: 8 row groups for single-k-step convs, else 4 (2 for NB >= 3) x up to 3
// ``half``: half the row groups in flight (fewer VGPRs -> more waves per SIMD; an autotuner candidate, cfg bit 10)
template <int NB>
void direct_launch_nb(const ConvParams& p, int rpb, bool epi, bool half, hipStream_t s) {
  const int KS = direct_ks(p);
  if (half) {
    if (KS == 1) direct_launch_cfg<NB, (NB <= 2 ? 4 : 2), 1>(p, rpb, epi, s);
    else if (KS == 2) direct_launch_cfg<NB, (NB <= 2 ? 2 : 1), 2>(p, rpb, epi, s);
    else direct_launch_cfg<NB, (NB <= 2 ? 2 : 1), 3>(p, rpb, epi, s);
    return;
  }
  if (KS == 1) direct_launch_cfg<NB, (NB <= 2 ? 8 : 4), 1>(p, rpb, epi, s);
  else if (KS == 2) direct_launch_cfg<NB, (NB <= 2 ? 4 : 2), 2>(p, rpb, epi, s);
  else direct_launch_cfg<NB, (NB <= 2 ? 4 : 2), 3>(p, rpb, epi, s);
}

}  // namespace

// rows per workgroup of configuration word cfg (bit 5 set = direct kernel; bit 6: 2048 rows, else 512)
int conv_direct_rows(int cfg) { return (cfg & 64) ? 2048 : 512; }

// 1 when the direct kernel can run this launch: 16-B chunks, <= 64 output channels, weights fit in LDS
int conv_direct_legal(const ConvParams& p, int chunk) {
  if (chunk != 8 || p.Ngemm > 64 || p.Cg % 8 != 0) return 0;
  if (p.nt * p.nh * p.nw == 0) return 0;
  const int NB = (p.Ngemm + 15) / 16;
  return direct_lds(p, NB) <= 80 * 1024 ? 1 : 0;   // >= 2 workgroups per CU (160 KB LDS)
}

void conv_direct_launch(const ConvParams& p, int cfg, hipStream_t s) {
  const int rpb = conv_direct_rows(cfg);
  const bool epi = p.eres || p.emask || p.epart;
  const bool half = (cfg & 1024) != 0;
  switch ((p.Ngemm + 15) / 16) {
    case 1: direct_launch_nb<1>(p, rpb, epi, half, s); break;
    case 2: direct_launch_nb<2>(p, rpb, epi, half, s); break;
    case 3: direct_launch_nb<3>(p, rpb, epi, half, s); break;
    default: direct_launch_nb<4>(p, rpb, epi, half, s); break;
  }
}

PVA_NS_END  // namespace PVA_NS
