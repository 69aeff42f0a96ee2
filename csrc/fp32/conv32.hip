// fp32 convolutions for gfx950 on split-bf16 MFMA (the "--mixed_precision no" path; reference run.py:330 default).
//
// Every fp32 operand is split while it is staged into LDS into NP bf16 pieces, x = p0 + p1 [+ p2] (p0 = bf16(x) RNE,
// p1 = bf16(x - p0), p2 = bf16(x - p0 - p1)), and each MFMA 16x16x32 fragment pair issues the products whose order is
// above the target precision, into one fp32 accumulator:
//   NP = 3 ("bf16x6", default): p0p0 + p0p1 + p1p0 + p0p2 + p2p0 + p1p1 — operands carry 24 bits, dropped terms are
//          <= 2^-24 relative: fp32 accuracy at a sixth of the bf16 MFMA rate (~415 TF/s peak);
//   NP = 2 ("bf16x3"): p0p0 + p0p1 + p1p0 — ~16-bit operands (2^-16 relative per product) at a third of the rate.
// Both beat gfx950's f32-input MFMA (157 TF/s, MI355X_MICROARCH.md "matrix cores") on throughput.
//
// LDS image of a tile: NP planes, plane p = [rows][64 B] holding piece p of 32 k values as four 16-B chunks, chunk c
// stored at chunk c ^ ((row >> 1) & 3) — conflict-free for the ds_read_b128 fragment reads (lane l reads row l & 15,
// chunk l >> 4) under gfx950's 4 x 16-lane grouping.
//
// igemm32: implicit GEMM over positions (forward, and each stride phase of the input gradient: csrc/fp32/f32_params.h),
//   register-staged LDS (double-buffered at NP = 2: one barrier per 32-k step), swapped MFMA operands so each lane
//   owns 4 consecutive output channels (16-B stores).
// wgrad32: weight gradient, positions on the reduction axis (split across workgroups, fp32 atomics): both operands
//   are staged transposed (each loading thread holds 8 positions x 4 channels and writes one 16-B chunk per channel
//   and piece); half the threads load the gathered input, half the output gradient.
#include "../kernels/common.h"
#include "f32_params.h"

namespace pva_f32 {

template <int NP>
__device__ __forceinline__ void split4(const float4& v, uint2 (&o)[NP]) {
  float r0 = v.x, r1 = v.y, r2 = v.z, r3 = v.w;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const uint32_t a = cvt_pk_e16(r0, r1), b = cvt_pk_e16(r2, r3);
    o[p] = make_uint2(a, b);
    if (p + 1 < NP) {
      r0 -= lo2f(a);
      r1 -= hi2f(a);
      r2 -= lo2f(b);
      r3 -= hi2f(b);
    }
  }
}

template <int NP>
__device__ __forceinline__ void split8(float (&f)[8], uint4 (&o)[NP]) {
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[i] = cvt_pk_e16(f[2 * i], f[2 * i + 1]);
      if (p + 1 < NP) {
        f[2 * i] -= lo2f(w[i]);
        f[2 * i + 1] -= hi2f(w[i]);
      }
    }
    o[p] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// n / d for 0 <= n < 2^31 with the host-computed (m, s) of magic_div
__device__ __forceinline__ int fdiv(int n, unsigned m, int s) {
  return (int)((__umulhi((unsigned)n, m) + (unsigned)n) >> s);
}
static void magic_div(int d, unsigned* m, int* s) {
  int k = 0;
  while ((1LL << k) < d) ++k;
  *s = k;
  *m = (unsigned)((((1ULL << 32) * ((1ULL << k) - (unsigned long long)d)) / (unsigned long long)d + 1) & 0xffffffffULL);
}

__device__ __forceinline__ int chunk_off(int r, int c) { return r * 64 + ((c ^ ((r >> 1) & 3)) << 4); }

__device__ __forceinline__ float4 affine4(float4 v, const float4& s, const float4& h, int relu) {
  v.x = fmaf(v.x, s.x, h.x);
  v.y = fmaf(v.y, s.y, h.y);
  v.z = fmaf(v.z, s.z, h.z);
  v.w = fmaf(v.w, s.w, h.w);
  if (relu) {
    v.x = fmaxf(v.x, 0.f);
    v.y = fmaxf(v.y, 0.f);
    v.z = fmaxf(v.z, 0.f);
    v.w = fmaxf(v.w, 0.f);
  }
  return v;
}

#define PVA_MF(x, y, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(ev8_t, x), __builtin_bit_cast(ev8_t, y), c, 0, 0, 0)

// One 32-k step of a wave's (16 FM) x (16 FN) sub-tile: D[n][m] += B[n][:] . A[m][:] over the split pieces.
// sA / sB: plane 0 of the A (rowsA rows) / B (rowsB rows) images; plane p is p * rows * 64 bytes further.
template <int NP, int FM, int FN>
__device__ __forceinline__ void mma_split(const uint8_t* sA, int rowsA, const uint8_t* sB, int rowsB, int ra, int rb,
                                          int lane, f32x4_t (&acc)[FM][FN]) {
  const int g = lane >> 4, l15 = lane & 15;
  uint4 b[NP][FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int o = chunk_off(rb + 16 * j + l15, g);
#pragma unroll
    for (int p = 0; p < NP; ++p) b[p][j] = *reinterpret_cast<const uint4*>(sB + p * rowsB * 64 + o);
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    uint4 a[NP];
    const int o = chunk_off(ra + 16 * i + l15, g);
#pragma unroll
    for (int p = 0; p < NP; ++p) a[p] = *reinterpret_cast<const uint4*>(sA + p * rowsA * 64 + o);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      f32x4_t c = acc[i][j];
      // smallest terms first
      if constexpr (NP == 3) {
        c = PVA_MF(b[1][j], a[1], c);
        c = PVA_MF(b[2][j], a[0], c);
        c = PVA_MF(b[0][j], a[2], c);
      }
      c = PVA_MF(b[1][j], a[0], c);
      c = PVA_MF(b[0][j], a[1], c);
      c = PVA_MF(b[0][j], a[0], c);
      acc[i][j] = c;
    }
  }
}

// A operand loads go through a buffer resource rebased to the first clip this tile's rows read (32-bit offsets, no
// 64-bit address math): per row, the position part of the offset is fixed for the whole k loop (VGPR) and the tap +
// channel part is wave-uniform (SGPR soffset) when the k-step lies inside one tap (UNI: Cr % 32 == 0); an
// out-of-range tap position or a row past M gets an offset past the resource, which loads zeros in hardware.  B rows
// are the pre-split weight planes (wpack32: piece p of row n at p * wplane + n * ldw), stored to LDS as loaded.
template <int NP, int BM, int BN, int WGM, bool UNI>
__global__ __launch_bounds__(256) void igemm32_kernel(const Conv32 p) {
  constexpr int WGN = 4 / WGM, TM = BM / WGM, TN = BN / WGN, FM = TM / 16, FN = TN / 16;
  constexpr int LA = (BM + 31) / 32, LB = (BN + 31) / 32;
  constexpr int NBUF = NP == 2 ? 2 : 1;   // NP = 3 images are 1.5x larger: one buffer, two barriers per step
  constexpr int IMG = NP * (BM + BN) * 64;
  constexpr unsigned OOB = 0x80000000u;
  static_assert(FM >= 1 && FN >= 1 && TM % 16 == 0 && TN % 16 == 0, "wave tile");
  __shared__ __attribute__((aligned(16))) uint8_t smem[NBUF][IMG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WGM, wn = wave / WGM;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kq = tid & 7, r0 = tid >> 3;
  const int HWi = p.Hi * p.Wi;
  const int Q = p.Qt * p.Qh * p.Qw;
  const int64_t clip = (int64_t)p.Ti * HWi * p.ldx;   // elements per input clip
  const int nbf = m0 / Q, nbl = min(m0 + BM - 1, p.M - 1) / Q;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.x + nbf * clip), (short)0, (int)((nbl - nbf + 1) * clip * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, 3 * p.wplane * 2,
                                                                      0x00020000);
  // per A row: position offset in bytes (channel quad kq included) and the tap-free input coordinates
  unsigned aoff[LA];
  int at[LA], ahh[LA], aww[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int r = r0 + 32 * i, m = m0 + r;
    const bool ok = r < BM && m < p.M;
    int mm = ok ? m : 0;
    const int qw = mm % p.Qw;
    mm /= p.Qw;
    const int qh = mm % p.Qh;
    mm /= p.Qh;
    const int qt = mm % p.Qt, nb = mm / p.Qt;
    at[i] = ok ? qt * p.st : -(1 << 20);   // a row past M fails every bounds test
    ahh[i] = qh * p.sh;
    aww[i] = qw * p.sw;
    aoff[i] = (unsigned)((((int64_t)(nb - nbf) * p.Ti * HWi + (int64_t)at[i] * HWi + ahh[i] * p.Wi + aww[i]) * p.ldx +
                          4 * kq) * 4);
  }
  unsigned boff[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int r = r0 + 32 * i, n = n0 + r;
    boff[i] = (r < BN && n < p.N) ? (unsigned)((n * p.ldw + 4 * kq) * 2) : OOB;
  }
  f32x4_t ra[LA];
  uint2 rb[LB][NP];
  const int nk = (p.K + 31) / 32;
  const f32x4_t z4 = {0.f, 0.f, 0.f, 0.f};
  int tj = 0, tc = 0;   // UNI: tap index and channel base of the next k-step to load (wave-uniform)

  auto load = [&](int kt) {
    int dt, dh, dw, widx, c;   // c: this lane's first channel (UNI: + 4 kq is inside aoff)
    bool kv = true;
    if constexpr (UNI) {
      const int4 tp = reinterpret_cast<const int4*>(p.taps)[tj];
      dt = tp.x; dh = tp.y; dw = tp.z; widx = tp.w;
      c = tc;
      tc += 32;
      if (tc == p.Cr) { tc = 0; ++tj; }
    } else {
      const int k = kt * 32 + 4 * kq;
      kv = k < p.K;
      const int j = kv ? k / p.Cr : 0;
      c = k - j * p.Cr - 4 * kq;
      const int4 tp = reinterpret_cast<const int4*>(p.taps)[j];
      dt = tp.x; dh = tp.y; dw = tp.z; widx = tp.w;
    }
    const int toff = ((dt * p.Hi + dh) * p.Wi + dw) * p.ldx + c;   // elements
    f32x4_t sc = z4, sh = z4;
    const bool aff = p.isc != nullptr;
    if (aff) {
      sc = *reinterpret_cast<const f32x4_t*>(p.isc + c + 4 * kq);
      sh = *reinterpret_cast<const f32x4_t*>(p.ish + c + 4 * kq);
    }
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const bool ok = kv && (unsigned)(at[i] + dt) < (unsigned)p.Ti && (unsigned)(ahh[i] + dh) < (unsigned)p.Hi &&
                      (unsigned)(aww[i] + dw) < (unsigned)p.Wi;
      // (the whole offset in the VGPR: the hardware range check does not cover a negative tap offset in soffset)
      f32x4_t v = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                  xr, ok ? aoff[i] + (unsigned)(toff * 4) : OOB, 0, 0));
      if (aff) {
        v = v * sc + sh;
        if (p.irelu) v = __builtin_elementwise_max(v, z4);
        v = ok ? v : z4;   // padding stays zero after the transform
      }
      ra[i] = v;
    }
    const int wk = (widx * p.Cr + c) * 2;   // bytes
#pragma unroll
    for (int i = 0; i < LB; ++i)
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const unsigned o = UNI ? boff[i] : (kv ? boff[i] + wk : OOB);
        rb[i][q] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(wr, o, (UNI ? wk : 0) + q * p.wplane * 2, 0));
      }
  };
  auto store = [&](uint8_t* img) {
    const int hc = kq >> 1, ho = (kq & 1) << 3;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int r = r0 + 32 * i;
      if (r < BM) {
        uint2 o[NP];
        split4<NP>(float4{ra[i][0], ra[i][1], ra[i][2], ra[i][3]}, o);
        const int off = chunk_off(r, hc) + ho;
#pragma unroll
        for (int q = 0; q < NP; ++q) *reinterpret_cast<uint2*>(img + q * BM * 64 + off) = o[q];
      }
    }
    uint8_t* imgB = img + NP * BM * 64;
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int r = r0 + 32 * i;
      if (r < BN) {
        const int off = chunk_off(r, hc) + ho;
#pragma unroll
        for (int q = 0; q < NP; ++q) *reinterpret_cast<uint2*>(imgB + q * BN * 64 + off) = rb[i][q];
      }
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  load(0);
  for (int kt = 0; kt < nk; ++kt) {
    uint8_t* img = smem[NBUF == 2 ? (kt & 1) : 0];
    if (NBUF == 1 && kt > 0) __syncthreads();   // every wave is done reading the previous step
    store(img);
    __syncthreads();
    if (kt + 1 < nk) load(kt + 1);
    mma_split<NP, FM, FN>(img, BM, img + NP * BM * 64, BN, wm * TM, wn * TN, lane, acc);
  }

  if (p.stats != nullptr) {   // per-tile channel sums of y and y^2 (BatchNorm statistics, no re-read of y)
    float* red = reinterpret_cast<float*>(&smem[0][0]);   // [WGM][2][BN]
    __syncthreads();                                      // every wave is done with the last step's image
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < FM; ++i)
          if (m0 + wm * TM + 16 * i + (lane & 15) < p.M) {
            const float v = acc[i][j][r];
            s1 += v;
            s2 = fmaf(v, v, s2);
          }
        s1 = sum16(s1);
        s2 = sum16(s2);
        if ((lane & 15) == 0) {
          const int nl = wn * TN + 16 * j + 4 * (lane >> 4) + r;
          red[(wm * 2) * BN + nl] = s1;
          red[(wm * 2 + 1) * BN + nl] = s2;
        }
      }
    __syncthreads();
    for (int t = tid; t < 2 * BN; t += 256) {
      const int q = t / BN, nl = t - q * BN;
      if (n0 + nl >= p.N) continue;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < WGM; ++w) v += red[(w * 2 + q) * BN + nl];
      p.stats[((int64_t)blockIdx.x * 2 + q) * p.N + n0 + nl] = v;
    }
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm * TM + 16 * i + (lane & 15);
    if (m >= p.M) continue;
    int mm = m;
    const int qw = mm % p.Qw;
    mm /= p.Qw;
    const int qh = mm % p.Qh;
    mm /= p.Qh;
    const int qt = mm % p.Qt, nb = mm / p.Qt;
    const int64_t row = (((int64_t)nb * p.Yt + qt * p.ost + p.ort) * p.Yh + qh * p.osh + p.orh) * p.Yw +
                        qw * p.osw + p.orw;
    float* yr = p.y + row * p.ldy;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * TN + 16 * j + 4 * (lane >> 4);
      if (n < p.N) {
        float4 v = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        if (p.accum) {
          const float4 o = *reinterpret_cast<const float4*>(yr + n);
          v.x += o.x;
          v.y += o.y;
          v.z += o.z;
          v.w += o.w;
        }
        *reinterpret_cast<float4*>(yr + n) = v;
      }
    }
  }
}

// channel E of 8 staged positions -> NP split pieces, one 16-B chunk each, into row r of a transposed image
template <int NP, int E>
__device__ __forceinline__ void store_comp(const f32x4_t (&rv)[8], uint8_t* base, int rows, int r, int po) {
  float f[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) f[u] = rv[u][E];
  uint4 o[NP];
  split8<NP>(f, o);
  const int off = chunk_off(r, po);
#pragma unroll
  for (int k = 0; k < NP; ++k) *reinterpret_cast<uint4*>(base + k * rows * 64 + off) = o[k];
}

// Weight gradient.  A rows = k = (tap, cin) (BM per tile), B rows = cout (BN per tile); D[cout][k] so the 16 lanes of
// a fragment column hold consecutive k (coalesced atomics).  Stages of 32 positions; threads [0, BM) load the
// gathered input (BM/4 channel quads x 4 position octets), threads [BM, BM + BN) the output gradient.
template <int NP, int BM, int BN, int WGM>
__global__ __launch_bounds__(256) void wgrad32_kernel(const Wgrad32 p) {
  constexpr int WGN = 4 / WGM, TM = BM / WGM, TN = BN / WGN, FM = TM / 16, FN = TN / 16;
  constexpr int QA = BM / 4, QB = BN / 4;
  static_assert(FM >= 1 && FN >= 1 && BM + BN <= 256, "tile");
  __shared__ __attribute__((aligned(16))) uint8_t smem[NP * (BM + BN) * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WGM, wn = wave / WGM;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int p_begin = blockIdx.z * p.chunk;
  const int p_end = min(p.P, p_begin + p.chunk);
  if (p_begin >= p_end) return;
  const f32x4_t z4 = {0.f, 0.f, 0.f, 0.f};   // native vectors: a select of HIP's float4 struct goes through scratch
  const bool xr = tid < BM;                          // gathered-input role
  const bool dr = tid >= BM && tid < BM + BN;        // output-gradient role
  const int lt = xr ? tid : tid - BM;
  const int q = xr ? lt % QA : lt % QB, po = xr ? lt / QA : lt / QB;   // channel quad, position octet (0..3)
  const int kk = m0 + 4 * q;
  const bool kkv = xr && kk < p.K;
  int xc = 0, tdt = 0, tdh = 0, tdw = 0;
  if (kkv) {
    const int j = kk / p.Cin;
    xc = kk - j * p.Cin;
    tdt = p.taps[4 * j];
    tdh = p.taps[4 * j + 1];
    tdw = p.taps[4 * j + 2];
  }
  const int dn = n0 + 4 * q;
  const bool dnv = dr && dn < p.Cout;
  const int HWi = p.Hi * p.Wi;

  f32x4_t rv[8];
  auto load = [&](int s0) {
    const int pos = s0 + 8 * po;
    // loads are unconditional from a valid address (a predicated "cond ? *ptr : 0" becomes a flat load through a
    // pointer select with a zero in scratch); out-of-range values are zeroed afterwards
    if (dr) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool ok = dnv && pos + u < p_end;
        const f32x4_t v = *reinterpret_cast<const f32x4_t*>(p.dy + (ok ? (int64_t)(pos + u) * p.ldd + dn : 0));
        rv[u] = ok ? v : z4;
      }
      return;
    }
    const bool aff = kkv && p.isc != nullptr;
    const f32x4_t isc = *reinterpret_cast<const f32x4_t*>(aff ? p.isc + xc : p.x);   // (always a global address)
    const f32x4_t ish = *reinterpret_cast<const f32x4_t*>(aff ? p.ish + xc : p.x);
    const int m0p = pos < p_end ? pos : 0;
    const int m1 = fdiv(m0p, p.mqw, p.sqw), m2 = fdiv(m1, p.mqh, p.sqh);
    int qw = m0p - m1 * p.Qw, qh = m1 - m2 * p.Qh;
    int nb = fdiv(m2, p.mqt, p.sqt), qt = m2 - nb * p.Qt;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      {
        const int ti = qt * p.st + tdt, hi = qh * p.sh + tdh, wi = qw * p.sw + tdw;
        const bool ok = kkv && pos + u < p_end && (unsigned)ti < (unsigned)p.Ti && (unsigned)hi < (unsigned)p.Hi &&
                        (unsigned)wi < (unsigned)p.Wi;
        f32x4_t v = *reinterpret_cast<const f32x4_t*>(
            p.x + (ok ? ((int64_t)nb * p.Ti * HWi + (int64_t)ti * HWi + hi * p.Wi + wi) * p.ldx + xc : 0));
        if (aff) {
          v = v * isc + ish;
          if (p.irelu) v = __builtin_elementwise_max(v, z4);
        }
        rv[u] = ok ? v : z4;
      }
      // next position: branch-free carry (keeps the loop unrolled and rv[] in registers)
      ++qw;
      const bool c1 = qw == p.Qw;
      qw = c1 ? 0 : qw;
      qh += c1;
      const bool c2 = qh == p.Qh;
      qh = c2 ? 0 : qh;
      qt += c2;
      const bool c3 = qt == p.Qt;
      qt = c3 ? 0 : qt;
      nb += c3;
    }
  };
  auto store = [&]() {
    if (!xr && !dr) return;
    uint8_t* base = xr ? smem : smem + NP * BM * 64;
    const int rows = xr ? BM : BN;
    store_comp<NP, 0>(rv, base, rows, 4 * q + 0, po);
    store_comp<NP, 1>(rv, base, rows, 4 * q + 1, po);
    store_comp<NP, 2>(rv, base, rows, 4 * q + 2, po);
    store_comp<NP, 3>(rv, base, rows, 4 * q + 3, po);
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  load(p_begin);
  for (int s0 = p_begin; s0 < p_end; s0 += 32) {
    if (s0 != p_begin) __syncthreads();
    store();
    __syncthreads();
    if (s0 + 32 < p_end) load(s0 + 32);
    mma_split<NP, FM, FN>(smem, BM, smem + NP * BM * 64, BN, wm * TM, wn * TN, lane, acc);
  }
  // D[cout][k]: lane column = k (lane & 15), rows = cout 4*(lane>>4) + r
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int k = m0 + wm * TM + 16 * i + (lane & 15);
    if (k >= p.K) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * TN + 16 * j + 4 * (lane >> 4);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (n + r < p.Cout) unsafeAtomicAdd(p.dw + (int64_t)(n + r) * p.ldw + k, acc[i][j][r]);
    }
  }
}

// ---------------------------------------------------------------- weight layouts
// the three bf16 pieces of an fp32 weight (the same split as split4<3>), one per plane
__device__ __forceinline__ void put_split3(uint16_t* dst, int64_t i, int64_t plane, float v) {
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const uint32_t b = cvt_pk_e16(v, 0.f);
    dst[q * plane + i] = (uint16_t)(b & 0xffffu);
    v -= lo2f(b);
  }
}

// torch w[co][ci][tap] -> forward B rows wf[piece][co][tap][cip] (zero channels ci >= Cin)
__global__ void wpack_fwd_kernel(const float* w, uint16_t* wf, int Cout, int Cin, int taps, int cip) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n = (int64_t)Cout * taps * cip;
  if (i >= n) return;
  const int c = i % cip;
  const int64_t t = i / cip;
  const int tap = t % taps, co = t / taps;
  put_split3(wf, i, n, c < Cin ? w[((int64_t)co * Cin + c) * taps + tap] : 0.f);
}

// torch w[co][ci][tap] -> input-gradient B rows wt[piece][ci][tap][co]
__global__ void wpack_dgrad_kernel(const float* w, uint16_t* wt, int Cout, int Cin, int taps) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n = (int64_t)Cout * taps * Cin;
  if (i >= n) return;
  const int co = i % Cout;
  const int64_t t = i / Cout;
  const int tap = t % taps, ci = t / taps;
  put_split3(wt, i, n, w[((int64_t)co * Cin + ci) * taps + tap]);
}

// wgrad layout dwf[co][tap][cip] -> torch g[co][ci][tap] (= beta*g + value)
__global__ void wunpack_kernel(const float* dwf, float* g, int Cout, int Cin, int taps, int cip, float beta) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n = (int64_t)Cout * Cin * taps;
  if (i >= n) return;
  const int tap = i % taps;
  const int64_t t = i / taps;
  const int ci = t % Cin, co = t / Cin;
  const float v = dwf[((int64_t)co * taps + tap) * cip + ci];
  g[i] = beta != 0.f ? fmaf(beta, g[i], v) : v;
}

// ---------------------------------------------------------------- host launchers
template <int NP, int BM, int BN, int WGM>
static void igemm_go(const Conv32& p, hipStream_t s) {
  dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN);
  if (p.Cr % 32 == 0) hipLaunchKernelGGL((igemm32_kernel<NP, BM, BN, WGM, true>), grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((igemm32_kernel<NP, BM, BN, WGM, false>), grid, dim3(256), 0, s, p);
}

int igemm32_tile(int N) { return N > 64 ? 0 : N > 32 ? 1 : N > 16 ? 2 : 3; }
int igemm32_bm(int N) { return igemm32_tile(N) == 3 ? 256 : 128; }

template <int NP>
static void igemm_np(const Conv32& p, hipStream_t s) {
  switch (igemm32_tile(p.N)) {
    case 0: igemm_go<NP, 128, 128, 2>(p, s); break;
    case 1: igemm_go<NP, 128, 64, 2>(p, s); break;
    case 2: igemm_go<NP, 128, 32, 4>(p, s); break;
    default: igemm_go<NP, 256, 16, 4>(p, s); break;
  }
}

void igemm32_launch(const Conv32& p, int np, hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return;
  if (np == 2) igemm_np<2>(p, s);
  else igemm_np<3>(p, s);
}

template <int NP, int BM, int BN, int WGM>
static void wgrad_go(const Wgrad32& p, int splits, hipStream_t s) {
  dim3 grid((p.K + BM - 1) / BM, (p.Cout + BN - 1) / BN, splits);
  hipLaunchKernelGGL((wgrad32_kernel<NP, BM, BN, WGM>), grid, dim3(256), 0, s, p);
}

static int tile_of(int n) { return n > 64 ? 128 : n > 32 ? 64 : n > 16 ? 32 : 16; }

// workgroup tile (k rows x cout rows) for a weight gradient
void wgrad32_tile(int K, int Cout, int* bm, int* bn) {
  int a = tile_of(K), b = tile_of(Cout);
  if (a * b < 1024) {  // a 4-wave tile needs >= 16x16 per wave
    if (a < b) a = 1024 / b; else b = 1024 / a;
  }
  *bm = a;
  *bn = b;
}

template <int NP>
static void wgrad_np(const Wgrad32& p, int bm, int bn, int splits, hipStream_t s) {
#define PVA_W32(A, B, G) \
  if (bm == A && bn == B) return wgrad_go<NP, A, B, G>(p, splits, s);
  PVA_W32(128, 128, 2) PVA_W32(128, 64, 2) PVA_W32(64, 128, 2) PVA_W32(64, 64, 2) PVA_W32(128, 32, 4)
  PVA_W32(32, 128, 1) PVA_W32(128, 16, 4) PVA_W32(16, 128, 1) PVA_W32(64, 32, 2) PVA_W32(32, 64, 2)
  PVA_W32(64, 16, 4) PVA_W32(16, 64, 1) PVA_W32(32, 32, 2)
#undef PVA_W32
}

void wgrad32_launch(Wgrad32 p, int np, hipStream_t s) {
  if (p.P <= 0 || p.K <= 0 || p.Cout <= 0) return;
  int bm, bn;
  wgrad32_tile(p.K, p.Cout, &bm, &bn);
  const int tiles = ((p.K + bm - 1) / bm) * ((p.Cout + bn - 1) / bn);
  const int stages = (p.P + 31) / 32;
  int splits = (2048 + tiles - 1) / tiles;
  splits = splits < 1 ? 1 : splits > stages ? stages : splits;
  p.chunk = ((stages + splits - 1) / splits) * 32;
  splits = (p.P + p.chunk - 1) / p.chunk;
  magic_div(p.Qw, &p.mqw, &p.sqw);
  magic_div(p.Qh, &p.mqh, &p.sqh);
  magic_div(p.Qt, &p.mqt, &p.sqt);
  if (np == 2) wgrad_np<2>(p, bm, bn, splits, s);
  else wgrad_np<3>(p, bm, bn, splits, s);
}

void wpack32_launch(int mode, const float* src, void* dst, int Cout, int Cin, int taps, int cip, float beta,
                    hipStream_t s) {
  const int64_t n = mode == 1 ? (int64_t)Cout * taps * Cin : mode == 0 ? (int64_t)Cout * taps * cip
                                                                       : (int64_t)Cout * Cin * taps;
  if (n == 0) return;
  const int blocks = (int)((n + 255) / 256);
  if (mode == 0)
    hipLaunchKernelGGL(wpack_fwd_kernel, dim3(blocks), dim3(256), 0, s, src, (uint16_t*)dst, Cout, Cin, taps, cip);
  else if (mode == 1)
    hipLaunchKernelGGL(wpack_dgrad_kernel, dim3(blocks), dim3(256), 0, s, src, (uint16_t*)dst, Cout, Cin, taps);
  else
    hipLaunchKernelGGL(wunpack_kernel, dim3(blocks), dim3(256), 0, s, src, (float*)dst, Cout, Cin, taps, cip, beta);
}

}  // namespace pva_f32
