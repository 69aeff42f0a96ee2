// fp32 convolutions for gfx950 on bf16x3 MFMA (the "--mixed_precision no" path; reference run.py:330 default).
//
// Every fp32 operand is split while it is staged into LDS: hi = bf16(x) (RNE), lo = bf16(x - hi).  Each MFMA
// 16x16x32 fragment pair then issues three products into one fp32 accumulator: hi*hi + hi*lo + lo*hi (the lo*lo term,
// 2^-16 relative, is dropped).  That is ~fp32 accuracy at a third of the bf16 MFMA rate (~830 TF/s peak), against
// 157 TF/s for gfx950's f32-input MFMA (MI355X_MICROARCH.md, matrix cores).
//
// LDS image of a tile: one 128-B row per GEMM row holding 32 k values as eight 16-B chunks (chunks 0-3: hi of k
// 8c..8c+7, chunks 4-7: lo), chunk c stored at chunk c ^ (row & 7) — conflict-free for the ds_read_b128 fragment
// reads (lane l reads row l&15, chunk l>>4) under gfx950's 4 x 16-lane grouping.
//
// igemm32: implicit GEMM over positions (forward, and each stride phase of the input gradient: csrc/fp32/f32_params.h),
//   register-staged double-buffered LDS, one barrier per 32-k step, swapped MFMA operands so each lane owns 4
//   consecutive output channels (16-B stores).
// wgrad32: weight gradient, positions on the reduction axis (split across workgroups, fp32 atomics): both operands
//   are staged transposed (each thread loads 8 positions x 4 channels and writes one 16-B chunk per channel).
#include "../kernels/common.h"
#include "f32_params.h"

namespace pva_f32 {

__device__ __forceinline__ void split4(const float4& v, uint2& hi, uint2& lo) {
  const uint32_t h0 = cvt_pk_e16(v.x, v.y), h1 = cvt_pk_e16(v.z, v.w);
  hi = make_uint2(h0, h1);
  lo = make_uint2(cvt_pk_e16(v.x - lo2f(h0), v.y - hi2f(h0)), cvt_pk_e16(v.z - lo2f(h1), v.w - hi2f(h1)));
}

__device__ __forceinline__ void split8(const float* f, uint4& hi, uint4& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h[i] = cvt_pk_e16(f[2 * i], f[2 * i + 1]);
    l[i] = cvt_pk_e16(f[2 * i] - lo2f(h[i]), f[2 * i + 1] - hi2f(h[i]));
  }
  hi = make_uint4(h[0], h[1], h[2], h[3]);
  lo = make_uint4(l[0], l[1], l[2], l[3]);
}

__device__ __forceinline__ int chunk_off(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }

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

// One 32-k step of a wave's (16 FM) x (16 FN) sub-tile: D[n][m] += B[n][:] . A[m][:] in bf16x3.
template <int FM, int FN>
__device__ __forceinline__ void mma3(const uint8_t* sA, const uint8_t* sB, int ra, int rb, int lane,
                                     f32x4_t (&acc)[FM][FN]) {
  const int g = lane >> 4, l15 = lane & 15;
  uint4 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int r = ra + 16 * i + l15;
    ah[i] = *reinterpret_cast<const uint4*>(sA + chunk_off(r, g));
    al[i] = *reinterpret_cast<const uint4*>(sA + chunk_off(r, 4 + g));
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int r = rb + 16 * j + l15;
    bh[j] = *reinterpret_cast<const uint4*>(sB + chunk_off(r, g));
    bl[j] = *reinterpret_cast<const uint4*>(sB + chunk_off(r, 4 + g));
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const ev8_t bhv = __builtin_bit_cast(ev8_t, bh[j]), blv = __builtin_bit_cast(ev8_t, bl[j]);
      const ev8_t ahv = __builtin_bit_cast(ev8_t, ah[i]), alv = __builtin_bit_cast(ev8_t, al[i]);
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(blv, ahv, acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bhv, alv, acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bhv, ahv, acc[i][j], 0, 0, 0);
    }
  }
}

template <int BM, int BN, int WGM>
__global__ __launch_bounds__(256) void igemm32_kernel(const Conv32 p) {
  constexpr int WGN = 4 / WGM, TM = BM / WGM, TN = BN / WGN, FM = TM / 16, FN = TN / 16;
  constexpr int LA = (BM + 31) / 32, LB = (BN + 31) / 32;
  static_assert(FM >= 1 && FN >= 1 && TM % 16 == 0 && TN % 16 == 0, "wave tile");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2][(BM + BN) * 128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WGM, wn = wave / WGM;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kq = tid & 7, r0 = tid >> 3;
  const int HWi = p.Hi * p.Wi;
  int64_t abase[LA];
  int at[LA], ahh[LA], aww[LA];
  bool aval[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int r = r0 + 32 * i, m = m0 + r;
    aval[i] = r < BM && m < p.M;
    int mm = aval[i] ? m : 0;
    const int qw = mm % p.Qw;
    mm /= p.Qw;
    const int qh = mm % p.Qh;
    mm /= p.Qh;
    const int qt = mm % p.Qt, nb = mm / p.Qt;
    abase[i] = (int64_t)nb * p.Ti * HWi;
    at[i] = qt * p.st;
    ahh[i] = qh * p.sh;
    aww[i] = qw * p.sw;
  }
  float4 ra[LA], rb[LB];
  const int nk = (p.K + 31) / 32;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);

  auto load = [&](int kt) {
    const int k = kt * 32 + 4 * kq;
    const bool kv = k < p.K;
    int c = 0;
    int4 tp = make_int4(0, 0, 0, 0);
    if (kv) {
      const int j = k / p.Cr;
      c = k - j * p.Cr;
      tp = reinterpret_cast<const int4*>(p.taps)[j];
    }
    float4 sc = z4, sh = z4;
    if (p.isc != nullptr && kv) {
      sc = *reinterpret_cast<const float4*>(p.isc + c);
      sh = *reinterpret_cast<const float4*>(p.ish + c);
    }
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      ra[i] = z4;
      if (kv && aval[i]) {
        const int ti = at[i] + tp.x, hi = ahh[i] + tp.y, wi = aww[i] + tp.z;
        if ((unsigned)ti < (unsigned)p.Ti && (unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi) {
          const float* src = p.x + (abase[i] + (int64_t)ti * HWi + hi * p.Wi + wi) * p.ldx + c;
          ra[i] = *reinterpret_cast<const float4*>(src);
          if (p.isc != nullptr) ra[i] = affine4(ra[i], sc, sh, p.irelu);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      rb[i] = z4;
      const int r = r0 + 32 * i, n = n0 + r;
      if (kv && r < BN && n < p.N)
        rb[i] = *reinterpret_cast<const float4*>(p.w + (int64_t)n * p.ldw + tp.w * p.Cr + c);
    }
  };
  auto store = [&](int buf) {
    uint8_t* sA = smem[buf];
    uint8_t* sB = smem[buf] + BM * 128;
    const int hc = kq >> 1, ho = (kq & 1) << 3;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int r = r0 + 32 * i;
      if (r < BM) {
        uint2 h, l;
        split4(ra[i], h, l);
        *reinterpret_cast<uint2*>(sA + chunk_off(r, hc) + ho) = h;
        *reinterpret_cast<uint2*>(sA + chunk_off(r, 4 + hc) + ho) = l;
      }
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int r = r0 + 32 * i;
      if (r < BN) {
        uint2 h, l;
        split4(rb[i], h, l);
        *reinterpret_cast<uint2*>(sB + chunk_off(r, hc) + ho) = h;
        *reinterpret_cast<uint2*>(sB + chunk_off(r, 4 + hc) + ho) = l;
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
    const int buf = kt & 1;
    store(buf);
    __syncthreads();
    if (kt + 1 < nk) load(kt + 1);
    mma3<FM, FN>(smem[buf], smem[buf] + BM * 128, wm * TM, wn * TN, lane, acc);
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

// Weight gradient.  sA rows = k = (tap, cin) (BM per tile), sB rows = cout (BN per tile); D[cout][k] so the 16 lanes
// of a fragment column hold consecutive k (coalesced atomics).
template <int BM, int BN, int WGM>
__global__ __launch_bounds__(256) void wgrad32_kernel(const Wgrad32 p) {
  constexpr int WGN = 4 / WGM, TM = BM / WGM, TN = BN / WGN, FM = TM / 16, FN = TN / 16;
  constexpr int QA = BM / 4, QB = BN / 4;
  static_assert(FM >= 1 && FN >= 1 && 8 * QA <= 256 && 8 * QB <= 256, "tile");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2][(BM + BN) * 128];  // two 32-position sub-steps
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WGM, wn = wave / WGM;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int p_begin = blockIdx.z * p.chunk;
  const int p_end = min(p.P, p_begin + p.chunk);
  if (p_begin >= p_end) return;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // X (gathered) role: rows k = m0 + 4*xq .. +3, positions 8*xpo .. +7 of each 64-position stage
  const bool xr = tid < 8 * QA;
  const int xq = tid % QA, xpo = tid / QA;
  const int kk = m0 + 4 * xq;
  const bool kkv = xr && kk < p.K;
  int xc = 0;
  int4 tp = make_int4(0, 0, 0, 0);
  if (kkv) {
    const int j = kk / p.Cin;
    xc = kk - j * p.Cin;
    tp = reinterpret_cast<const int4*>(p.taps)[j];
  }
  float4 isc = z4, ish = z4;
  if (kkv && p.isc != nullptr) {
    isc = *reinterpret_cast<const float4*>(p.isc + xc);
    ish = *reinterpret_cast<const float4*>(p.ish + xc);
  }
  // dY role: rows cout = n0 + 4*dq .. +3
  const bool dr = tid < 8 * QB;
  const int dq = tid % QB, dpo = tid / QB;
  const int dn = n0 + 4 * dq;
  const bool dnv = dr && dn < p.Cout;
  const int HWi = p.Hi * p.Wi;

  float4 rx[8], rd[8];
  auto load = [&](int s0) {
    {
      const int pos = s0 + 8 * dpo;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        rd[u] = (dnv && pos + u < p_end) ? *reinterpret_cast<const float4*>(p.dy + (int64_t)(pos + u) * p.ldd + dn)
                                         : z4;
    }
    const int pos = s0 + 8 * xpo;
    int mm = pos < p_end ? pos : 0;
    int qw = mm % p.Qw;
    mm /= p.Qw;
    int qh = mm % p.Qh;
    mm /= p.Qh;
    int qt = mm % p.Qt, nb = mm / p.Qt;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      rx[u] = z4;
      if (kkv && pos + u < p_end) {
        const int ti = qt * p.st + tp.x, hi = qh * p.sh + tp.y, wi = qw * p.sw + tp.z;
        if ((unsigned)ti < (unsigned)p.Ti && (unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi) {
          rx[u] = *reinterpret_cast<const float4*>(
              p.x + ((int64_t)nb * p.Ti * HWi + (int64_t)ti * HWi + hi * p.Wi + wi) * p.ldx + xc);
          if (p.isc != nullptr) rx[u] = affine4(rx[u], isc, ish, p.irelu);
        }
      }
      if (++qw == p.Qw) {
        qw = 0;
        if (++qh == p.Qh) {
          qh = 0;
          if (++qt == p.Qt) {
            qt = 0;
            ++nb;
          }
        }
      }
    }
  };
  auto store = [&]() {
    if (xr) {
      uint8_t* base = smem[xpo >> 2];
      const int cc = xpo & 3;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float f[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) f[u] = e == 0 ? rx[u].x : e == 1 ? rx[u].y : e == 2 ? rx[u].z : rx[u].w;
        uint4 h, l;
        split8(f, h, l);
        const int r = 4 * xq + e;
        *reinterpret_cast<uint4*>(base + chunk_off(r, cc)) = h;
        *reinterpret_cast<uint4*>(base + chunk_off(r, 4 + cc)) = l;
      }
    }
    if (dr) {
      uint8_t* base = smem[dpo >> 2] + BM * 128;
      const int cc = dpo & 3;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float f[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) f[u] = e == 0 ? rd[u].x : e == 1 ? rd[u].y : e == 2 ? rd[u].z : rd[u].w;
        uint4 h, l;
        split8(f, h, l);
        const int r = 4 * dq + e;
        *reinterpret_cast<uint4*>(base + chunk_off(r, cc)) = h;
        *reinterpret_cast<uint4*>(base + chunk_off(r, 4 + cc)) = l;
      }
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  load(p_begin);
  for (int s0 = p_begin; s0 < p_end; s0 += 64) {
    __syncthreads();
    store();
    __syncthreads();
    if (s0 + 64 < p_end) load(s0 + 64);
    mma3<FM, FN>(smem[0], smem[0] + BM * 128, wm * TM, wn * TN, lane, acc);
    mma3<FM, FN>(smem[1], smem[1] + BM * 128, wm * TM, wn * TN, lane, acc);
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
// torch w[co][ci][tap] -> forward B rows wf[co][tap][cip] (zero channels ci >= Cin)
__global__ void wpack_fwd_kernel(const float* w, float* wf, int Cout, int Cin, int taps, int cip) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n = (int64_t)Cout * taps * cip;
  if (i >= n) return;
  const int c = i % cip;
  const int64_t t = i / cip;
  const int tap = t % taps, co = t / taps;
  wf[i] = c < Cin ? w[((int64_t)co * Cin + c) * taps + tap] : 0.f;
}

// torch w[co][ci][tap] -> input-gradient B rows wt[ci][tap][co]
__global__ void wpack_dgrad_kernel(const float* w, float* wt, int Cout, int Cin, int taps) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n = (int64_t)Cout * taps * Cin;
  if (i >= n) return;
  const int co = i % Cout;
  const int64_t t = i / Cout;
  const int tap = t % taps, ci = t / taps;
  wt[i] = w[((int64_t)co * Cin + ci) * taps + tap];
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
template <int BM, int BN, int WGM>
static void igemm_go(const Conv32& p, hipStream_t s) {
  dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN);
  hipLaunchKernelGGL((igemm32_kernel<BM, BN, WGM>), grid, dim3(256), 0, s, p);
}

int igemm32_tile(int N) { return N > 64 ? 0 : N > 32 ? 1 : N > 16 ? 2 : 3; }

void igemm32_launch(const Conv32& p, hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return;
  switch (igemm32_tile(p.N)) {
    case 0: igemm_go<128, 128, 2>(p, s); break;
    case 1: igemm_go<128, 64, 2>(p, s); break;
    case 2: igemm_go<128, 32, 4>(p, s); break;
    default: igemm_go<256, 16, 4>(p, s); break;
  }
}

template <int BM, int BN, int WGM>
static void wgrad_go(const Wgrad32& p, int splits, hipStream_t s) {
  dim3 grid((p.K + BM - 1) / BM, (p.Cout + BN - 1) / BN, splits);
  hipLaunchKernelGGL((wgrad32_kernel<BM, BN, WGM>), grid, dim3(256), 0, s, p);
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

void wgrad32_launch(Wgrad32 p, hipStream_t s) {
  if (p.P <= 0 || p.K <= 0 || p.Cout <= 0) return;
  int bm, bn;
  wgrad32_tile(p.K, p.Cout, &bm, &bn);
  const int tiles = ((p.K + bm - 1) / bm) * ((p.Cout + bn - 1) / bn);
  const int stages = (p.P + 63) / 64;
  int splits = (2048 + tiles - 1) / tiles;
  splits = splits < 1 ? 1 : splits > stages ? stages : splits;
  p.chunk = ((stages + splits - 1) / splits) * 64;
  splits = (p.P + p.chunk - 1) / p.chunk;
#define PVA_W32(A, B, G) \
  if (bm == A && bn == B) return wgrad_go<A, B, G>(p, splits, s);
  PVA_W32(128, 128, 2) PVA_W32(128, 64, 2) PVA_W32(64, 128, 2) PVA_W32(64, 64, 2) PVA_W32(128, 32, 4)
  PVA_W32(32, 128, 1) PVA_W32(128, 16, 4) PVA_W32(16, 128, 1) PVA_W32(64, 32, 2) PVA_W32(32, 64, 2)
  PVA_W32(64, 16, 4) PVA_W32(16, 64, 1) PVA_W32(32, 32, 2)
#undef PVA_W32
}

void wpack32_launch(int mode, const float* src, float* dst, int Cout, int Cin, int taps, int cip, float beta,
                    hipStream_t s) {
  const int64_t n = mode == 1 ? (int64_t)Cout * taps * Cin : mode == 0 ? (int64_t)Cout * taps * cip
                                                                       : (int64_t)Cout * Cin * taps;
  if (n == 0) return;
  const int blocks = (int)((n + 255) / 256);
  if (mode == 0)
    hipLaunchKernelGGL(wpack_fwd_kernel, dim3(blocks), dim3(256), 0, s, src, dst, Cout, Cin, taps, cip);
  else if (mode == 1)
    hipLaunchKernelGGL(wpack_dgrad_kernel, dim3(blocks), dim3(256), 0, s, src, dst, Cout, Cin, taps);
  else
    hipLaunchKernelGGL(wunpack_kernel, dim3(blocks), dim3(256), 0, s, src, dst, Cout, Cin, taps, cip, beta);
}

}  // namespace pva_f32
