// Fused backward of a narrow 1x1 conv whose BatchNorm is not folded (the fast pathway's res2 conv_c, 8 -> 32 channels
// at 16M positions per step at B=160, and the first unit's branch1, whose input is an activation: no affine, no mask,
// gradient accumulated into dx).  One streaming pass replaces three:
//
//   BN-backward apply   dyc = A*dz + B*yc + C          dz = g (masked by the unit's ReLU bits)
//   weight gradient     dWc[c][k] += dyc[c] * act_b[k]     act_b = relu(yb*sb + hb) (BN_b + ReLU recompute)
//   input gradient      v[k] = sum_c dyc[c] Wc[c][k], masked by act_b > 0; BN_b backward partial sums of v
//   identity shortcut   dz itself into dx (optional, written or accumulated)
//
// so dyc (the widest tensor of the unit's backward) is never written to HBM and read back twice.  The per-element
// arithmetic follows the unfused kernels: dyc rounded to the 16-bit type (as the apply stored it), act_b rounded
// after the affine (as the weight-gradient loader staged it), dab rounded before its partial sums (as the dgrad
// epilogue did).
//
// Layout: LPR = CO / 8 lanes per row, each owning 8 output channels c (16-B loads of g / yc / dz); every lane keeps
// the 8 x CI partial weight gradient of its channels in registers over the workgroup's row range, and the 8 x CI
// slice of Wc.  The per-row dgrad partials are summed over the row's lanes with DPP adds; lane q then finishes
// input channels k = q*CI/LPR .. (q+1)*CI/LPR - 1 (mask, round, store, partial sums).  Workgroup w owns rows
// [w*rps, (w+1)*rps): its weight-gradient slab and BN partial sums are written once, summed in a fixed order by the
// slab reduction / BN finalize (bitwise reproducible).
#include "common.h"

PVA_NS_BEGIN

namespace {

struct NarrowBwdParams {
  const uint16_t* g;      // [M][ldg] unit-output gradient (already masked when mode == 0)
  const uint8_t* mask;    // mode 3: ReLU bits [M][CO/8]
  const uint16_t* yc;     // raw conv output [M][CO] (BN input)
  const float* coef;      // BN backward coefficients [A | B | C] x CO
  uint16_t* dz;           // optional identity-shortcut gradient out [M][lddz]
  const uint16_t* yb;     // conv input [M][CI]: raw conv_b output (aff: BN_b + ReLU applied here) or an activation
  const float* sb;        // aff: BN_b scale / shift (forward affine)
  const float* hb;
  const float* mb;        // aff: BN_b batch mean / rstd (partial-sum rebase)
  const float* rb;
  const uint16_t* wc;     // packed conv weights [CO][CI]
  uint16_t* dab;          // [M][ldo] input gradient (aff: masked by the BN_b ReLU); accum: added to it
  float* slab;            // [splits][CO][CI] weight-gradient partials
  float* part;            // aff: [splits][3][CI] BN_b partial sums (sum v, sum v*xhat_b, 0)
  // reduce pass of a folded unit (no yc in memory): BN_c / BN_1 backward partial sums [splits][3][CO]
  const uint16_t* y1;     // branch1 raw output (its BN shares dz) or null
  const float* mc;        // BN_c batch mean / rstd, BN_1 batch mean / rstd
  const float* rc;
  const float* m1;
  const float* r1;
  float* cpart;
  int64_t M;
  int ldg, lddz, dz_accum, mode, rps, aff, accum, ldo;
};

// RC: the BN_c input yc is recomputed from act_b (yc[c] = sum_k Wc[c][k] act_b[k], rounded like the stored output)
// instead of read — the unit's conv_c is BN-folded in the forward (fold_output writes the unit output directly; yc
// never exists).  RED: the reduce pass of such a unit — only the BN_c (and BN_1) backward partial sums.
template <int CO, int CI, bool RC, bool RED>
__global__ __launch_bounds__(256) void narrow_c_bwd_kernel(const NarrowBwdParams p) {
  constexpr int LPR = CO / 8;            // lanes per row
  constexpr int RPW = 64 / LPR;          // rows per wave and pass
  constexpr int KPL = CI / LPR;          // input channels finished per lane
  static_assert(CO % 8 == 0 && 64 % LPR == 0 && CI % LPR == 0 && CI == 8, "narrow_c_bwd: CO 8..64, CI 8");
  __shared__ float red[4][LPR][8 * CI + 2 * CI];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int q = lane % LPR, rr = lane / LPR;
  const int c0 = 8 * q;
  const bool aff = p.aff != 0;
  // loop-invariant operands in registers (2 waves per SIMD; measured: staging them in LDS for 3 waves per SIMD made
  // the pass 25 % slower — 26 dependent LDS reads per row)
  float A[8], B[8], Cc[8], W[8][CI], sb[CI], hb[CI];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    A[e] = p.coef[c0 + e];
    B[e] = p.coef[CO + c0 + e];
    Cc[e] = p.coef[2 * CO + c0 + e];
#pragma unroll
    for (int k = 0; k < CI; ++k) W[e][k] = e2f(p.wc[(c0 + e) * CI + k]);
  }
#pragma unroll
  for (int k = 0; k < CI; ++k) { sb[k] = aff ? p.sb[k] : 1.f; hb[k] = aff ? p.hb[k] : 0.f; }
  float acc[8][CI];
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int k = 0; k < CI; ++k) acc[e][k] = 0.f;
  float sv[KPL], sy[KPL];
#pragma unroll
  for (int j = 0; j < KPL; ++j) { sv[j] = 0.f; sy[j] = 0.f; }

  const int64_t r_begin = (int64_t)blockIdx.x * p.rps;
  const int64_t r_end = r_begin + p.rps < p.M ? r_begin + p.rps : p.M;
  constexpr int STEP = 4 * RPW;
  // raw operands of the NEXT row are loaded one iteration ahead (software pipelining: a wave keeps two rows of
  // loads in flight at 2 waves per SIMD)
  uint4 ng{}, nc{}, nb{}, n1{};
  unsigned nbits = 0xffu;
  const bool dual = RED && p.y1 != nullptr;
  auto fetch = [&](int64_t r) {
    if (r < r_end) {
      ng = *reinterpret_cast<const uint4*>(p.g + r * p.ldg + c0);
      if constexpr (!RC) nc = *reinterpret_cast<const uint4*>(p.yc + r * CO + c0);
      nb = *reinterpret_cast<const uint4*>(p.yb + r * CI);
      if (dual) n1 = *reinterpret_cast<const uint4*>(p.y1 + r * CO + c0);
      if (p.mode == 3) nbits = p.mask[r * (CO / 8) + q];
    }
  };
  float rs[8], rsc[8], rs1[8];   // RED: sum dz, sum dz*yc, sum dz*y1 (raw; rebased at the end)
#pragma unroll
  for (int e = 0; e < 8; ++e) { rs[e] = 0.f; rsc[e] = 0.f; rs1[e] = 0.f; }
  int64_t r = r_begin + w * RPW + rr;
  fetch(r);
  for (; r < r_end; r += STEP) {
    float gz[8], yc[8], yb[CI], y1v[8];
    unpack8(ng, gz);
    if constexpr (!RC) unpack8(nc, yc);
    unpack8(nb, yb);
    if (dual) unpack8(n1, y1v);
    const unsigned bits = nbits;
    fetch(r + STEP);
    if (p.mode == 3) {
#pragma unroll
      for (int e = 0; e < 8; ++e) gz[e] = (bits >> e) & 1u ? gz[e] : 0.f;
    }
    // act_b = relu(BN_b(yb)) as the weight-gradient loader stages it (affine, round, ReLU); or yb itself
    float ab[CI];
    if (aff) {
      float t[CI];
#pragma unroll
      for (int k = 0; k < CI; ++k) t[k] = __builtin_fmaf(yb[k], sb[k], hb[k]);
      unpack8(relu_e16x8(pack8_fast(t)), ab);
    } else {
#pragma unroll
      for (int k = 0; k < CI; ++k) ab[k] = yb[k];
    }
    if constexpr (RC) {   // the folded forward's conv_c output, rounded as a stored output would be
      float t[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float a_ = 0.f;
#pragma unroll
        for (int k = 0; k < CI; ++k) a_ = __builtin_fmaf(W[e][k], ab[k], a_);
        t[e] = a_;
      }
      unpack8(pack8(t), yc);
    }
    if constexpr (RED) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        rs[e] += gz[e];
        rsc[e] = __builtin_fmaf(gz[e], yc[e], rsc[e]);
        if (dual) rs1[e] = __builtin_fmaf(gz[e], y1v[e], rs1[e]);
      }
      continue;
    }
    if (p.dz) {
      uint16_t* d = p.dz + r * p.lddz + c0;
      float o[8] = {gz[0], gz[1], gz[2], gz[3], gz[4], gz[5], gz[6], gz[7]};
      if (p.dz_accum) {
        float x[8];
        unpack8(*reinterpret_cast<const uint4*>(d), x);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += x[e];
      }
      *reinterpret_cast<uint4*>(d) = pack8(o);
    }
    // dyc, rounded to the compute type (the unfused apply stored it so)
    float dy[8];
    {
      float t[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) t[e] = A[e] * gz[e] + B[e] * yc[e] + Cc[e];
      unpack8(pack8(t), dy);
    }
    float pd[CI];
#pragma unroll
    for (int k = 0; k < CI; ++k) pd[k] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int k = 0; k < CI; ++k) {
        acc[e][k] = __builtin_fmaf(dy[e], ab[k], acc[e][k]);
        pd[k] = __builtin_fmaf(dy[e], W[e][k], pd[k]);
      }
    // sum the row's LPR lanes (adjacent lanes, DPP): every lane ends with the row's full dgrad
#pragma unroll
    for (int k = 0; k < CI; ++k) pd[k] = sum_lanes<LPR>(pd[k]);
    // lane q: input channels k = q*KPL + j — BN_b ReLU mask (affine of yb > 0), round, store, partial sums
    uint16_t* dst = p.dab + r * p.ldo + q * KPL;
    float old[KPL];
#pragma unroll
    for (int j = 0; j < KPL; ++j) old[j] = 0.f;
    if (p.accum) {
#pragma unroll
      for (int j = 0; j < KPL; ++j) old[j] = e2f(dst[j]);
    }
    float v[KPL];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
      const int k = q * KPL + j;
      float pk = 0.f, yk = 0.f, sk = 0.f, hk = 0.f;
#pragma unroll
      for (int kk = 0; kk < CI; ++kk)
        if (kk == k) { pk = pd[kk]; yk = yb[kk]; sk = sb[kk]; hk = hb[kk]; }
      v[j] = pk + old[j];
      if (aff) v[j] = (yk * sk + hk) > 0.f ? v[j] : 0.f;
      v[j] = e2f(f2e(v[j]));
      sv[j] += v[j];
      sy[j] += v[j] * yk;
    }
    if constexpr (KPL == 2) {
      *reinterpret_cast<uint32_t*>(dst) = cvt_pk_e16(v[0], v[1]);
    } else {
#pragma unroll
      for (int j = 0; j < KPL; ++j) dst[j] = f2e(v[j]);
    }
  }
  if constexpr (RED) {
    // lanes of the same channel group q (stride LPR), then the 4 waves in a fixed order
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1) {
        rs[e] += __shfl_xor(rs[e], o, 64);
        rsc[e] += __shfl_xor(rsc[e], o, 64);
        rs1[e] += __shfl_xor(rs1[e], o, 64);
      }
    float* rr3 = &red[0][0][0];   // [4 waves][3][CO]
    if (rr == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        rr3[(w * 3 + 0) * CO + c0 + e] = rs[e];
        rr3[(w * 3 + 1) * CO + c0 + e] = rsc[e];
        rr3[(w * 3 + 2) * CO + c0 + e] = rs1[e];
      }
    }
    __syncthreads();
    if (tid < CO) {
      const int c = tid;
      float t[3];
#pragma unroll
      for (int k = 0; k < 3; ++k)
        t[k] = ((rr3[(0 * 3 + k) * CO + c] + rr3[(1 * 3 + k) * CO + c]) + rr3[(2 * 3 + k) * CO + c]) +
               rr3[(3 * 3 + k) * CO + c];
      float* pt = p.cpart + (int64_t)blockIdx.x * 3 * CO;
      pt[c] = t[0];
      pt[CO + c] = (t[1] - p.mc[c] * t[0]) * p.rc[c];
      pt[2 * CO + c] = dual ? (t[2] - p.m1[c] * t[0]) * p.r1[c] : 0.f;
    }
    return;
  }
  // weight gradient: lanes of the same channel group q (stride LPR) -> one value per (c, k) per wave
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int k = 0; k < CI; ++k) {
      float t = acc[e][k];
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1) t += __shfl_xor(t, o, 64);
      acc[e][k] = t;
    }
#pragma unroll
  for (int j = 0; j < KPL; ++j)
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1) {
      sv[j] += __shfl_xor(sv[j], o, 64);
      sy[j] += __shfl_xor(sy[j], o, 64);
    }
  if (rr == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int k = 0; k < CI; ++k) red[w][q][e * CI + k] = acc[e][k];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
      red[w][q][8 * CI + j] = sv[j];
      red[w][q][8 * CI + CI + j] = sy[j];
    }
  }
  __syncthreads();
  float* slab = p.slab + (int64_t)blockIdx.x * CO * CI;
  for (int i = tid; i < CO * CI; i += 256) {
    const int c = i / CI, k = i - c * CI;
    const int qq = c / 8, e = c - qq * 8;
    slab[i] = ((red[0][qq][e * CI + k] + red[1][qq][e * CI + k]) + red[2][qq][e * CI + k]) + red[3][qq][e * CI + k];
  }
  if (aff && tid < CI) {
    const int k = tid, qq = k / KPL, j = k - qq * KPL;
    const float s = ((red[0][qq][8 * CI + j] + red[1][qq][8 * CI + j]) + red[2][qq][8 * CI + j]) + red[3][qq][8 * CI + j];
    const float y = ((red[0][qq][9 * CI + j] + red[1][qq][9 * CI + j]) + red[2][qq][9 * CI + j]) +
                    red[3][qq][9 * CI + j];
    float* pt = p.part + (int64_t)blockIdx.x * 3 * CI;
    pt[k] = s;
    pt[CI + k] = (y - p.mb[k] * s) * p.rb[k];
    pt[2 * CI + k] = 0.f;
  }
}

}  // namespace

int narrow_c_bwd_legal(int CO, int CI) { return (CO == 32 || CO == 16 || CO == 64) && CI == 8; }

// rows per workgroup (multiple of one pass of 4 waves) for a split count near `splits`
int narrow_c_bwd_rps(int64_t M, int CO, int splits) {
  const int pass = 4 * (64 / (CO / 8));
  int64_t rps = (M + splits - 1) / splits;
  rps = (rps + pass - 1) / pass * pass;
  return (int)(rps < pass ? pass : rps);
}

template <int CO>
static void narrow_launch_co(const NarrowBwdParams& p, int form, int grid, hipStream_t s) {
  if (form == 2) hipLaunchKernelGGL((narrow_c_bwd_kernel<CO, 8, true, true>), dim3(grid), dim3(256), 0, s, p);
  else if (form == 1) hipLaunchKernelGGL((narrow_c_bwd_kernel<CO, 8, true, false>), dim3(grid), dim3(256), 0, s, p);
  else hipLaunchKernelGGL((narrow_c_bwd_kernel<CO, 8, false, false>), dim3(grid), dim3(256), 0, s, p);
}

// form 0: yc read; 1: yc recomputed (folded unit); 2: reduce pass of a folded unit (cpart only)
void narrow_c_bwd_launch(const uint16_t* g, int ldg, int mode, const uint8_t* mask, const uint16_t* yc,
                         const float* coef, uint16_t* dz, int lddz, int dz_accum, const uint16_t* yb, const float* sb,
                         const float* hb, const float* mb, const float* rb, const uint16_t* wc, uint16_t* dab, int ldo,
                         int accum, float* slab, float* part, const uint16_t* y1, const float* mc, const float* rc,
                         const float* m1, const float* r1, float* cpart, int form, int64_t M, int CO, int CI, int rps,
                         hipStream_t s) {
  NarrowBwdParams p{g,  mask, yc, coef, dz,   yb,  sb,       hb,   mb,  rb,  wc,  dab, slab, part, y1, mc, rc, m1, r1,
                    cpart, M, ldg, lddz, dz_accum, mode, rps, sb != nullptr ? 1 : 0, accum, ldo};
  const int grid = (int)((M + rps - 1) / rps);
  if (grid <= 0) return;
  switch (CO) {
    case 16: narrow_launch_co<16>(p, form, grid, s); break;
    case 64: narrow_launch_co<64>(p, form, grid, s); break;
    default: narrow_launch_co<32>(p, form, grid, s); break;
  }
}

PVA_NS_END  // namespace PVA_NS
