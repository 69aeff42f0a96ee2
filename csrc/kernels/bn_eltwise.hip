// Training-mode BatchNorm3d + ReLU + residual + pooling kernels for NDHWC bf16 activations (gfx950).
//
// The conv epilogue already produced per-tile (sum, sumsq) partial slabs of each raw conv output y;
// bn_finalize turns them into batch statistics, updates running stats (momentum, unbiased var) and
// emits the per-channel affine (scale, shift) that consumers apply on load.  Everything elementwise
// is 16-B vectorised (8 channels per lane, cdna_hip_programming.md Guideline 13) and works on strided
// channel views (ld = row stride) so concatenated tensors are never copied.
//
// Backward: bn_bwd_reduce computes deterministic per-block partial sums of dz = g*mask, dz*xhat for
// up to two BN inputs sharing one dz (conv_c and branch1 of a residual unit), bn_bwd_finalize turns
// them into dgamma/dbeta (into the fp32 master-gradient buffer) and the coefficients of
//   dy = A*dz + B*y + C            (A = g*r, B = -g*r^2*dgamma/M, C = g*r*(mean*r*dgamma - dbeta)/M)
// and bn_bwd_apply materialises dy (bf16) for the dgrad/wgrad of the producing conv.
#include "common.h"
#include <algorithm>

PVA_NS_BEGIN

namespace {

constexpr int NT = 256;

// Thread -> (row lane lr, 8-channel vector c) mapping shared by the channel-vectorised kernels: the
// channel slot of a thread is fixed, so per-channel parameters are hoisted out of the row loop and no
// 64-bit division is needed per element.
#define ROW_VEC_SETUP(CH)                                  \
  const int vecs = (CH) >> 3;                              \
  const int rpi = NT / vecs;                               \
  const int lr = threadIdx.x / vecs;                       \
  const int c = (threadIdx.x - lr * vecs) << 3;            \
  if (lr >= rpi) return;

// ------------------------------------------------------------------------------------------
// finalize forward statistics
// ------------------------------------------------------------------------------------------
__global__ void bn_finalize_kernel(const float* __restrict__ part, int tiles, int C, int64_t count,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float* __restrict__ run_mean, float* __restrict__ run_var,
                                   int64_t* __restrict__ nbt, float momentum, float eps,
                                   float* __restrict__ save_mean, float* __restrict__ save_rstd,
                                   float* __restrict__ scale, float* __restrict__ shift) {
  const int c = blockIdx.x;
  double s = 0.0, q = 0.0;
  for (int t = threadIdx.x; t < tiles; t += NT) {
    s += part[(int64_t)t * 2 * C + c];
    q += part[(int64_t)t * 2 * C + C + c];
  }
  __shared__ double rs[NT], rq[NT];
  rs[threadIdx.x] = s; rq[threadIdx.x] = q;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) { rs[threadIdx.x] += rs[threadIdx.x + o]; rq[threadIdx.x] += rq[threadIdx.x + o]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double mean = rs[0] / (double)count;
    double var = rq[0] / (double)count - mean * mean;
    if (var < 0) var = 0;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    save_mean[c] = (float)mean;
    save_rstd[c] = rstd;
    const float g = gamma[c], b = beta[c];
    scale[c] = g * rstd;
    shift[c] = b - (float)mean * g * rstd;
    if (run_mean) {
      const double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unb;
    }
    if (c == 0 && nbt) nbt[0] += 1;
  }
}


// ---- two-level single-launch finalize (fwd and bwd share the reduction) -----------------------------------------
// The one-block-per-channel kernels above read a [tiles][K][C] slab with a 4-byte stride of K*C floats per thread:
// at 10^4-10^5 tiles that is ~100 dependent cache-line round trips per thread on C (often 8-64) workgroups.  Here
// grid = (C/64 channel groups) x S tile ranges: 256 threads = 64 channels x 4 tile lanes read whole 256-B rows
// (coalesced), each workgroup's double partials go to its own scratch row, and the LAST workgroup of a channel group
// to finish (agent-scope acq_rel counter, reset to 0 for the next use) sums the S partials in a fixed order and
// finalizes: bitwise deterministic, one launch, all CUs busy.
constexpr int FIN_TILES_PER_BLOCK = 64;

__device__ __forceinline__ bool fin_reduce_and_elect(const float* __restrict__ part, int tiles, int C, int K, int k0,
                                                     int k1, double* __restrict__ scratch, unsigned* __restrict__ ctr,
                                                     double* red) {
  const int cl = threadIdx.x & 63, tl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int S = gridDim.y, sb = blockIdx.y;
  const int per = (tiles + S - 1) / S;
  const int t0 = sb * per, t1 = min(tiles, t0 + per);
  // four rows per tile lane in flight (independent accumulators, combined in a fixed order): the reduction is
  // latency-bound, one dependent load pair per iteration left most of each workgroup's time waiting
  double a = 0.0, b = 0.0;
  if (c < C) {
    double a4[4] = {0.0, 0.0, 0.0, 0.0}, b4[4] = {0.0, 0.0, 0.0, 0.0};
    int t = t0 + tl;
    for (; t + 12 < t1; t += 16) {
      float fa[4], fb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        fa[u] = part[((int64_t)(t + 4 * u) * K + k0) * C + c];
        fb[u] = part[((int64_t)(t + 4 * u) * K + k1) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { a4[u] += fa[u]; b4[u] += fb[u]; }
    }
    for (int u = 0; t < t1; t += 4, ++u) {
      a4[u & 3] += part[((int64_t)t * K + k0) * C + c];
      b4[u & 3] += part[((int64_t)t * K + k1) * C + c];
    }
    a = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    b = (b4[0] + b4[1]) + (b4[2] + b4[3]);
  }
  red[threadIdx.x] = a;
  red[NT + threadIdx.x] = b;
  __syncthreads();
  if (tl == 0 && c < C) {
    a = red[cl] + red[64 + cl] + red[128 + cl] + red[192 + cl];
    b = red[NT + cl] + red[NT + 64 + cl] + red[NT + 128 + cl] + red[NT + 192 + cl];
    scratch[((int64_t)sb * 2) * C + c] = a;
    scratch[((int64_t)sb * 2 + 1) * C + c] = b;
  }
  __syncthreads();   // every partial store of this workgroup issued and drained before the release below
  __shared__ int last;
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ctr + blockIdx.x, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == (unsigned)(S - 1);
    if (last) __hip_atomic_store(ctr + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return false;
  // the last workgroup: fixed-order sum of the S partials (tile lanes split the ranges, then a fixed 4-way sum)
  a = 0.0; b = 0.0;
  if (c < C) {
    double a4[4] = {0.0, 0.0, 0.0, 0.0}, b4[4] = {0.0, 0.0, 0.0, 0.0};
    int r = tl;
    for (; r + 12 < S; r += 16) {
      double fa[4], fb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        fa[u] = __builtin_nontemporal_load(scratch + ((int64_t)(r + 4 * u) * 2) * C + c);
        fb[u] = __builtin_nontemporal_load(scratch + ((int64_t)(r + 4 * u) * 2 + 1) * C + c);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { a4[u] += fa[u]; b4[u] += fb[u]; }
    }
    for (int u = 0; r < S; r += 4, ++u) {
      a4[u & 3] += __builtin_nontemporal_load(scratch + ((int64_t)r * 2) * C + c);
      b4[u & 3] += __builtin_nontemporal_load(scratch + ((int64_t)r * 2 + 1) * C + c);
    }
    a = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    b = (b4[0] + b4[1]) + (b4[2] + b4[3]);
  }
  red[threadIdx.x] = a;
  red[NT + threadIdx.x] = b;
  __syncthreads();
  if (tl == 0) {
    red[threadIdx.x] = red[cl] + red[64 + cl] + red[128 + cl] + red[192 + cl];
    red[NT + threadIdx.x] = red[NT + cl] + red[NT + 64 + cl] + red[NT + 128 + cl] + red[NT + 192 + cl];
  }
  return true;
}

__global__ void bn_finalize2_kernel(const float* __restrict__ part, int tiles, int C, int64_t count,
                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                    float* __restrict__ run_mean, float* __restrict__ run_var,
                                    int64_t* __restrict__ nbt, float momentum, float eps,
                                    float* __restrict__ save_mean, float* __restrict__ save_rstd,
                                    float* __restrict__ scale, float* __restrict__ shift,
                                    double* __restrict__ scratch, unsigned* __restrict__ ctr) {
  __shared__ double red[2 * NT];
  if (!fin_reduce_and_elect(part, tiles, C, 2, 0, 1, scratch, ctr, red)) return;
  const int cl = threadIdx.x;
  const int c = blockIdx.x * 64 + cl;
  if (cl >= 64 || c >= C) return;
  const double mean = red[cl] / (double)count;
  double var = red[NT + cl] / (double)count - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  save_mean[c] = (float)mean;
  save_rstd[c] = rstd;
  const float g = gamma[c], bb = beta[c];
  scale[c] = g * rstd;
  shift[c] = bb - (float)mean * g * rstd;
  if (run_mean) {
    const double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unb;
  }
  if (c == 0 && nbt) nbt[0] += 1;
}

__global__ void bn_bwd_finalize2_kernel(const float* __restrict__ part, int blocks, int C, int64_t count, int which,
                                        const float* __restrict__ gamma, const float* __restrict__ mean,
                                        const float* __restrict__ rstd, float* __restrict__ dgamma,
                                        float* __restrict__ dbeta, float beta_acc, float* __restrict__ coef,
                                        double* __restrict__ scratch, unsigned* __restrict__ ctr) {
  __shared__ double red[2 * NT];
  if (!fin_reduce_and_elect(part, blocks, C, 3, 0, 1 + which, scratch, ctr, red)) return;
  const int cl = threadIdx.x;
  const int c = blockIdx.x * 64 + cl;
  if (cl >= 64 || c >= C) return;
  const float db = (float)red[cl], dg = (float)red[NT + cl];
  if (dgamma) {
    dgamma[c] = (beta_acc == 0.f ? 0.f : beta_acc * dgamma[c]) + dg;
    dbeta[c] = (beta_acc == 0.f ? 0.f : beta_acc * dbeta[c]) + db;
  }
  const float gm = gamma[c], r = rstd[c], mu = mean[c];
  const float inv = 1.f / (float)count;
  coef[c] = gm * r;
  coef[C + c] = -gm * r * r * dg * inv;
  coef[2 * C + c] = gm * r * (mu * r * dg - db) * inv;
}

// eval-mode affine from running statistics
__global__ void bn_eval_affine_kernel(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                                      float eps, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float r = rsqrtf(rv[c] + eps);
  scale[c] = gamma[c] * r;
  shift[c] = beta[c] - rm[c] * gamma[c] * r;
}

// ------------------------------------------------------------------------------------------
// elementwise: out = act(y*scale + shift)       (strided channel views)
// ------------------------------------------------------------------------------------------
__global__ void bn_act_kernel(const uint16_t* __restrict__ y, int ldy, uint16_t* __restrict__ out, int ldo,
                              const float* __restrict__ scale, const float* __restrict__ shift, int relu,
                              int64_t M, int C) {
  ROW_VEC_SETUP(C);
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sc[e] = scale[c + e]; sh[e] = shift[c + e]; }
  for (int64_t m = (int64_t)blockIdx.x * rpi + lr; m < M; m += (int64_t)gridDim.x * rpi) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(y + m * ldy + c), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float z = f[e] * sc[e] + sh[e];
      f[e] = relu ? fmaxf(z, 0.f) : z;
    }
    *reinterpret_cast<uint4*>(out + m * ldo + c) = pack8(f);
  }
}

// residual unit output: out = relu(yc*sc + hc + (has_b1 ? y1*s1 + h1 : x))
__global__ void res_out_kernel(const uint16_t* __restrict__ yc, const float* __restrict__ sc, const float* __restrict__ hc,
                               const uint16_t* __restrict__ y1, const float* __restrict__ s1, const float* __restrict__ h1,
                               const uint16_t* __restrict__ x, int ldx, uint16_t* __restrict__ out, int ldo,
                               uint8_t* __restrict__ mask, int64_t M, int C) {
  ROW_VEC_SETUP(C);
  float a0[8], a1[8], b0[8], b1[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a0[e] = sc[c + e]; a1[e] = hc[c + e];
    b0[e] = y1 ? s1[c + e] : 1.f; b1[e] = y1 ? h1[c + e] : 0.f;
  }
  const uint16_t* sp = y1 ? y1 : x;
  const int lds = y1 ? C : ldx;
  for (int64_t m = (int64_t)blockIdx.x * rpi + lr; m < M; m += (int64_t)gridDim.x * rpi) {
    float a[8], b[8];
    unpack8(*reinterpret_cast<const uint4*>(yc + m * C + c), a);
    unpack8(*reinterpret_cast<const uint4*>(sp + m * lds + c), b);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = fmaxf(a[e] * a0[e] + a1[e] + b[e] * b0[e] + b1[e], 0.f);
    const uint4 pk = pack8(a);
    *reinterpret_cast<uint4*>(out + m * ldo + c) = pk;
    if (mask) {  // ReLU mask of the stored bf16 values: bit e of byte (m, c/8) = out[m][c+e] > 0
      const uint32_t w[4] = {pk.x, pk.y, pk.z, pk.w};
      uint32_t bits = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bits |= ((w[e] & 0x7fffu) != 0 && !(w[e] & 0x8000u)) ? 1u << (2 * e) : 0u;
        bits |= ((w[e] & 0x7fff0000u) != 0 && !(w[e] & 0x80000000u)) ? 1u << (2 * e + 1) : 0u;
      }
      mask[m * (C >> 3) + (c >> 3)] = (uint8_t)bits;
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward reductions
//   mask_mode 0: dz = g ; 1: dz = g * (mo > 0) ; 2: dz = g * (y0*ms + mh > 0) ;
//   3: dz = g * bit(mo)  (mo = uint8 ReLU mask bits [M][C/8] written by res_out)
// ------------------------------------------------------------------------------------------
template <int MM, bool Y0, bool Y1, bool DZ>
__global__ void bn_bwd_reduce_kernel(const uint16_t* __restrict__ g, int ldg,
                                     const void* __restrict__ mo_, int ldm,
                                     const float* __restrict__ ms, const float* __restrict__ mh,
                                     const uint16_t* __restrict__ y0, const float* __restrict__ mean0,
                                     const float* __restrict__ rstd0,
                                     const uint16_t* __restrict__ y1, const float* __restrict__ mean1,
                                     const float* __restrict__ rstd1,
                                     int64_t M, int C, int rows_per_block, float* __restrict__ part,
                                     uint16_t* __restrict__ dzout, int lddz) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [slots][3][C], NT*96 bytes
  const uint16_t* mo = static_cast<const uint16_t*>(mo_);
  const uint8_t* mb = static_cast<const uint8_t*>(mo_);
  const int vecs = C >> 3;
  const int rpi = NT / vecs;  // rows per iteration
  const int lv = threadIdx.x % vecs, lr = threadIdx.x / vecs;
  const int c = lv << 3;
  float sdz[8], s0[8], s1[8], m0[8], r0[8], m1[8], r1[8], MS[8], MH[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sdz[e] = 0.f; s0[e] = 0.f; s1[e] = 0.f; }
  if (lr < rpi) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      m0[e] = Y0 ? mean0[c + e] : 0.f; r0[e] = Y0 ? rstd0[c + e] : 0.f;
      m1[e] = Y1 ? mean1[c + e] : 0.f; r1[e] = Y1 ? rstd1[c + e] : 0.f;
      MS[e] = MM == 2 ? ms[c + e] : 0.f; MH[e] = MM == 2 ? mh[c + e] : 0.f;
    }
    const int64_t mbeg = (int64_t)blockIdx.x * rows_per_block;
    const int64_t mend = min<int64_t>(M, mbeg + rows_per_block);
    for (int64_t m = mbeg + lr; m < mend; m += rpi) {
      float dz[8], a[8];
      unpack8(*reinterpret_cast<const uint4*>(g + m * ldg + c), dz);
      if constexpr (Y0) unpack8(*reinterpret_cast<const uint4*>(y0 + m * C + c), a);
      else
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] = 0.f;
      if constexpr (MM == 1) {
        float o[8];
        unpack8(*reinterpret_cast<const uint4*>(mo + m * ldm + c), o);
#pragma unroll
        for (int e = 0; e < 8; ++e) dz[e] = o[e] > 0.f ? dz[e] : 0.f;
      } else if constexpr (MM == 3) {
        const unsigned bits = mb[m * ldm + (c >> 3)];
#pragma unroll
        for (int e = 0; e < 8; ++e) dz[e] = (bits >> e) & 1u ? dz[e] : 0.f;
      } else if constexpr (MM == 2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) dz[e] = (a[e] * MS[e] + MH[e]) > 0.f ? dz[e] : 0.f;
      }
      if constexpr (DZ) *reinterpret_cast<uint4*>(dzout + m * lddz + c) = pack8(dz);   // masked dz, same pass
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sdz[e] += dz[e];
        if constexpr (Y0) s0[e] += dz[e] * (a[e] - m0[e]) * r0[e];
      }
      if constexpr (Y1) {
        float b[8];
        unpack8(*reinterpret_cast<const uint4*>(y1 + m * C + c), b);
#pragma unroll
        for (int e = 0; e < 8; ++e) s1[e] += dz[e] * (b[e] - m1[e]) * r1[e];
      }
    }
  }
  // Deterministic block reduction (no float atomics): threads lv, lv+vecs, ... share channels.  With
  // vecs < 64 (power of two) a wave first reduces across its lanes and each wave owns one slot;
  // otherwise every row group lr owns a slot.  Slots are summed in a fixed order.
  const bool wred = vecs < 64 && (vecs & (vecs - 1)) == 0;
  if (wred) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sdz[e] = wave_sum_stride(sdz[e], vecs);
      s0[e] = wave_sum_stride(s0[e], vecs);
      s1[e] = wave_sum_stride(s1[e], vecs);
    }
  }
  const int nslots = wred ? NT / 64 : rpi;
  const int slot = wred ? (int)(threadIdx.x >> 6) : lr;
  if (lr < rpi && (!wred || (threadIdx.x & 63) < vecs)) {
    float* o = red + slot * 3 * C;
#pragma unroll
    for (int e = 0; e < 8; ++e) { o[c + e] = sdz[e]; o[C + c + e] = s0[e]; o[2 * C + c + e] = s1[e]; }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * C; i += NT) {
    float t = 0.f;
    for (int k = 0; k < nslots; ++k) t += red[k * 3 * C + i];
    part[(int64_t)blockIdx.x * 3 * C + i] = t;
  }
}

// per channel: sums over blocks -> dgamma/dbeta (grad buffers, accumulate with beta_acc) + apply coeffs
__global__ void bn_bwd_finalize_kernel(const float* __restrict__ part, int blocks, int C, int64_t count, int which,
                                       const float* __restrict__ gamma, const float* __restrict__ mean,
                                       const float* __restrict__ rstd, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta, float beta_acc, float* __restrict__ coef) {
  const int c = blockIdx.x;
  double sdz = 0.0, sx = 0.0;
  for (int t = threadIdx.x; t < blocks; t += NT) {
    sdz += part[(int64_t)t * 3 * C + c];
    sx += part[(int64_t)t * 3 * C + (1 + which) * C + c];
  }
  __shared__ double ra[NT], rb[NT];
  ra[threadIdx.x] = sdz; rb[threadIdx.x] = sx;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) { ra[threadIdx.x] += ra[threadIdx.x + o]; rb[threadIdx.x] += rb[threadIdx.x + o]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float db = (float)ra[0], dg = (float)rb[0];
    if (dgamma) {
      dgamma[c] = (beta_acc == 0.f ? 0.f : beta_acc * dgamma[c]) + dg;
      dbeta[c] = (beta_acc == 0.f ? 0.f : beta_acc * dbeta[c]) + db;
    }
    const float gm = gamma[c], r = rstd[c], mu = mean[c];
    const float inv = 1.f / (float)count;
    coef[c] = gm * r;                                   // A
    coef[C + c] = -gm * r * r * dg * inv;               // B
    coef[2 * C + c] = gm * r * (mu * r * dg - db) * inv;  // C
  }
}

// dy_k = A_k*dz + B_k*y_k + C_k  (k = 0, 1) ; optionally dz itself (identity shortcut gradient).
// Specialised at compile time on the mask mode and on which of y0 / y1 / dz take part: the common interior
// apply (no mask, y0 only) then needs ~1/2 of the registers of the all-modes kernel (116 VGPRs), i.e. twice
// the waves per SIMD to hide the latency of this streaming pass.
template <int MM, bool Y0, bool Y1, bool DZ>
__global__ void bn_bwd_apply_kernel(const uint16_t* __restrict__ g, int ldg,
                                    const void* __restrict__ mo_, int ldm,
                                    const float* __restrict__ ms, const float* __restrict__ mh,
                                    const uint16_t* __restrict__ y0, const float* __restrict__ coef0,
                                    uint16_t* __restrict__ dy0,
                                    const uint16_t* __restrict__ y1, const float* __restrict__ coef1,
                                    uint16_t* __restrict__ dy1,
                                    uint16_t* __restrict__ dzout, int lddz, int dz_accum,
                                    int64_t M, int C) {
  ROW_VEC_SETUP(C);
  const uint16_t* mo = static_cast<const uint16_t*>(mo_);
  const uint8_t* mb = static_cast<const uint8_t*>(mo_);
  float A0[8], B0[8], C0[8], A1[8], B1[8], C1[8], MS[8], MH[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if constexpr (Y0) { A0[e] = coef0[c + e]; B0[e] = coef0[C + c + e]; C0[e] = coef0[2 * C + c + e]; }
    if constexpr (Y1) { A1[e] = coef1[c + e]; B1[e] = coef1[C + c + e]; C1[e] = coef1[2 * C + c + e]; }
    if constexpr (MM == 2) { MS[e] = ms[c + e]; MH[e] = mh[c + e]; }
  }
  for (int64_t m = (int64_t)blockIdx.x * rpi + lr; m < M; m += (int64_t)gridDim.x * rpi) {
    float dz[8], a[8];
    unpack8(*reinterpret_cast<const uint4*>(g + m * ldg + c), dz);
    if constexpr (Y0) unpack8(*reinterpret_cast<const uint4*>(y0 + m * C + c), a);
    if constexpr (MM == 1) {
      float o[8];
      unpack8(*reinterpret_cast<const uint4*>(mo + m * ldm + c), o);
#pragma unroll
      for (int e = 0; e < 8; ++e) dz[e] = o[e] > 0.f ? dz[e] : 0.f;
    } else if constexpr (MM == 3) {
      const unsigned bits = mb[m * ldm + (c >> 3)];
#pragma unroll
      for (int e = 0; e < 8; ++e) dz[e] = (bits >> e) & 1u ? dz[e] : 0.f;
    } else if constexpr (MM == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) dz[e] = (a[e] * MS[e] + MH[e]) > 0.f ? dz[e] : 0.f;
    }
    float o[8];
    if constexpr (Y0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = A0[e] * dz[e] + B0[e] * a[e] + C0[e];
      *reinterpret_cast<uint4*>(dy0 + m * C + c) = pack8(o);
    }
    if constexpr (Y1) {
      float b[8];
      unpack8(*reinterpret_cast<const uint4*>(y1 + m * C + c), b);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = A1[e] * dz[e] + B1[e] * b[e] + C1[e];
      *reinterpret_cast<uint4*>(dy1 + m * C + c) = pack8(o);
    }
    if constexpr (DZ) {
      uint16_t* d = dzout + m * lddz + c;
      if (dz_accum) {
        float q[8];
        unpack8(*reinterpret_cast<const uint4*>(d), q);
#pragma unroll
        for (int e = 0; e < 8; ++e) dz[e] += q[e];
      }
      *reinterpret_cast<uint4*>(d) = pack8(dz);
    }
  }
}

// ------------------------------------------------------------------------------------------
// stem: out = maxpool_{1x3x3, s(1,2,2), p(0,1,1)}(relu(y*scale+shift)) ; argmax as 0..8 (uint8)
// ------------------------------------------------------------------------------------------
__global__ void stem_pool_fwd_kernel(const uint16_t* __restrict__ y, const float* __restrict__ scale,
                                     const float* __restrict__ shift, uint16_t* __restrict__ out,
                                     uint8_t* __restrict__ arg, uint16_t* __restrict__ ymax, int NT_, int H, int W,
                                     int Ho, int Wo, int C, int ldo) {
  // lane -> (pooled position, 8-channel vector); 32-bit index math (positions < 2^31, checked by the binding);
  // the 9 window loads are issued before any compare (independent loads in flight)
  ROW_VEC_SETUP(C);
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sc[e] = scale[c + e]; sh[e] = shift[c + e]; }
  const int Q = NT_ * Ho * Wo;
  for (int q = blockIdx.x * rpi + lr; q < Q; q += gridDim.x * rpi) {
    const int wo = q % Wo;
    const int r = q / Wo;
    const int ho = r % Ho;
    const int nt = r / Ho;
    uint4 v[9];
#pragma unroll
    for (int dh = 0; dh < 3; ++dh)
#pragma unroll
      for (int dw = 0; dw < 3; ++dw) {
        const int h = min(max(ho * 2 - 1 + dh, 0), H - 1), w = min(max(wo * 2 - 1 + dw, 0), W - 1);
        v[dh * 3 + dw] = *reinterpret_cast<const uint4*>(y + (((int64_t)nt * H + h) * W + w) * C + c);
      }
    float best[8], yb[8];
    uint32_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; yb[e] = 0.f; }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int h = ho * 2 - 1 + k / 3, w = wo * 2 - 1 + k % 3;
      if ((unsigned)h >= (unsigned)H || (unsigned)w >= (unsigned)W) continue;
      float f[8];
      unpack8(v[k], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float a = fmaxf(f[e] * sc[e] + sh[e], 0.f);
        if (a > best[e]) { best[e] = a; bi[e] = (uint32_t)k; yb[e] = f[e]; }
      }
    }
    const int64_t o = (int64_t)q * C + c;
    *reinterpret_cast<uint4*>(out + (int64_t)q * ldo + c) = pack8(best);
    uint2 pk;
    pk.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    pk.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    *reinterpret_cast<uint2*>(arg + o) = pk;
    if (ymax) *reinterpret_cast<uint4*>(ymax + o) = pack8(yb);   // raw conv output at the argmax (exact)
  }
}

// gather form of the max-pool backward: each input position sums the (<=4) windows whose argmax it is
__global__ void stem_pool_bwd_kernel(const uint16_t* __restrict__ dout, int ldd, const uint8_t* __restrict__ arg,
                                     uint16_t* __restrict__ dact, int NT_, int H, int W, int Ho, int Wo, int C) {
  const int vecs = C >> 3;
  const int64_t total = (int64_t)NT_ * H * W * vecs;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    int64_t r = i;
    const int cv = r % vecs; r /= vecs;
    const int w = r % W; r /= W;
    const int h = r % H; r /= H;
    const int64_t nt = r;
    const int c = cv << 3;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    // windows ho with ho*2-1 <= h <= ho*2+1
    const int ho_lo = (h) / 2, ho_hi = min(Ho - 1, (h + 1) / 2);
    const int wo_lo = (w) / 2, wo_hi = min(Wo - 1, (w + 1) / 2);
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      const int dh = h - (ho * 2 - 1);
      if (dh < 0 || dh > 2) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const int dw = w - (wo * 2 - 1);
        if (dw < 0 || dw > 2) continue;
        const int64_t o = (nt * Ho + ho) * Wo + wo;
        const uint2 pk = *reinterpret_cast<const uint2*>(arg + o * C + c);
        float g[8];
        unpack8(*reinterpret_cast<const uint4*>(dout + o * ldd + c), g);
        const uint8_t want = (uint8_t)(dh * 3 + dw);
        uint8_t bi[8] = {(uint8_t)(pk.x), (uint8_t)(pk.x >> 8), (uint8_t)(pk.x >> 16), (uint8_t)(pk.x >> 24),
                         (uint8_t)(pk.y), (uint8_t)(pk.y >> 8), (uint8_t)(pk.y >> 16), (uint8_t)(pk.y >> 24)};
#pragma unroll
        for (int e = 0; e < 8; ++e) if (bi[e] == want) acc[e] += g[e];
      }
    }
    *reinterpret_cast<uint4*>(dact + ((nt * H + h) * W + w) * C + c) = pack8(acc);
  }
}

// Stem backward, max-pool and BatchNorm fused.  dz (grad wrt relu(BN(y))) is non-zero only at window argmaxes,
// so the BN-backward sums sum(dz*mask), sum(dz*mask*xhat) are taken over the POOLED grid (bn_bwd_reduce on
// dout and the raw y at each argmax, ``ymax`` of stem_pool_fwd: 4x fewer bytes than the full-resolution dz),
// and this kernel produces dy = A*dz*mask + B*y + C in one pass: the argmax gather of dz, the ReLU mask from
// y's own affine and the BN apply — dz is never written.  Thread -> (position lane, 8-channel vector).
__global__ void stem_pool_bn_apply_kernel(const uint16_t* __restrict__ dout, int ldd, const uint8_t* __restrict__ arg,
                                          const uint16_t* __restrict__ y, const float* __restrict__ ms,
                                          const float* __restrict__ mh, const float* __restrict__ coef,
                                          uint16_t* __restrict__ dy, int NT_, int H, int W, int Ho, int Wo, int C) {
  // One lane owns the 2x2 input block (2ho+a, 2wo+b) of pooled window (ho, wo) for 8 channels.  Input row
  // 2ho+a lies in window ho (offset a+1) and, for a = 1, in window ho+1 (offset 0); likewise columns.  So
  // the four windows (ho..ho+1, wo..wo+1) are loaded once (unconditionally: independent loads in flight)
  // and serve all four positions.
  ROW_VEC_SETUP(C);
  float A[8], B[8], Cc[8], MS[8], MH[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    A[e] = coef[c + e]; B[e] = coef[C + c + e]; Cc[e] = coef[2 * C + c + e];
    MS[e] = ms[c + e]; MH[e] = mh[c + e];
  }
  const int Q = NT_ * Ho * Wo;   // < 2^31 (checked by the launcher)
  for (int q = blockIdx.x * rpi + lr; q < Q; q += gridDim.x * rpi) {
    const int wo = q % Wo;
    const int r = q / Wo;
    const int ho = r % Ho;
    const int nt = r / Ho;
    uint2 ag[2][2];
    float g[2][2][8];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool ok = ho + i < Ho && wo + j < Wo;
        const int64_t o = ((int64_t)nt * Ho + min(ho + i, Ho - 1)) * Wo + min(wo + j, Wo - 1);
        ag[i][j] = *reinterpret_cast<const uint2*>(arg + o * C + c);
        if (!ok) ag[i][j] = make_uint2(0xffffffffu, 0xffffffffu);   // matches no offset
        unpack8(*reinterpret_cast<const uint4*>(dout + o * ldd + c), g[i][j]);
      }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int h = 2 * ho + a;
      if (h >= H) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int w = 2 * wo + b;
        if (w >= W) continue;
        const int64_t m = ((int64_t)nt * H + h) * W + w;
        float yv[8], acc[8];
        unpack8(*reinterpret_cast<const uint4*>(y + m * C + c), yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
        for (int i = 0; i <= a; ++i)
#pragma unroll
          for (int j = 0; j <= b; ++j) {
            const uint32_t want = (uint32_t)((i ? 0 : a + 1) * 3 + (j ? 0 : b + 1));
            const uint2 pk = ag[i][j];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t bi = ((e < 4 ? pk.x : pk.y) >> (8 * (e & 3))) & 255u;
              acc[e] += bi == want ? g[i][j][e] : 0.f;
            }
          }
        float o8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dz = (yv[e] * MS[e] + MH[e]) > 0.f ? acc[e] : 0.f;
          o8[e] = A[e] * dz + B[e] * yv[e] + Cc[e];
        }
        *reinterpret_cast<uint4*>(dy + m * C + c) = pack8(o8);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Global average pool (window = the whole T x H x W volume, the SlowFast head at 224/256 crops):
// position-split partial sums [N][S][C] (16-B loads, 8 channels per lane, deterministic LDS reduction),
// then a fixed-order sum over the splits.  Backward is a pure 16-B broadcast store.
// ------------------------------------------------------------------------------------------
__global__ void avgpool_global_part_kernel(const uint16_t* __restrict__ x, int vol, int C, int S,
                                           float* __restrict__ part) {
  const int n = blockIdx.x / S, sp = blockIdx.x % S;
  const int vecs = C >> 3;
  const int rpi = NT / vecs;     // vecs <= NT (C <= 2048, checked by the launcher)
  const int lr = threadIdx.x / vecs;
  const int c = (threadIdx.x - lr * vecs) << 3;
  const int per = (vol + S - 1) / S;
  const int p0 = sp * per, p1 = min(vol, p0 + per);
  float s[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = 0.f;
  if (lr < rpi) {
    const uint16_t* base = x + (int64_t)n * vol * C + c;
    int p = p0 + lr;
    for (; p + 3 * rpi < p1; p += 4 * rpi) {   // 4 independent 16-B loads in flight per lane
      uint4 q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = *reinterpret_cast<const uint4*>(base + (int64_t)(p + k * rpi) * C);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float f[8];
        unpack8(q[k], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += f[e];
      }
    }
    for (; p < p1; p += rpi) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(base + (int64_t)p * C), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += f[e];
    }
  }
  __shared__ float red[NT * 8];
#pragma unroll
  for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = s[e];
  __syncthreads();
  for (int i = threadIdx.x; i < C; i += NT) {   // channel i = vector i/8, element i%8; rows in fixed order
    const int v = i >> 3, e = i & 7;
    float t = 0.f;
    for (int k = 0; k < rpi; ++k) t += red[(k * vecs + v) * 8 + e];
    part[((int64_t)n * S + sp) * C + i] = t;
  }
}

__global__ void avgpool_global_final_kernel(const float* __restrict__ part, int S, int C, float inv,
                                            float* __restrict__ out, int ldo, int coff, int N) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i % C;
  float t = 0.f;
  for (int k = 0; k < S; ++k) t += part[((int64_t)n * S + k) * C + c];
  out[(int64_t)n * ldo + coff + c] = t * inv;
}

__global__ void avgpool_global_bwd_kernel(const float* __restrict__ dout, int ldo, int coff, int vol, int C,
                                          float inv, uint16_t* __restrict__ dx, int64_t M) {
  ROW_VEC_SETUP(C);
  for (int64_t m = (int64_t)blockIdx.x * rpi + lr; m < M; m += (int64_t)gridDim.x * rpi) {
    const int64_t n = m / vol;
    const float4* src = reinterpret_cast<const float4*>(dout + n * ldo + coff + c);
    const float4 u = src[0], v = src[1];
    float f[8] = {u.x * inv, u.y * inv, u.z * inv, u.w * inv, v.x * inv, v.y * inv, v.z * inv, v.w * inv};
    *reinterpret_cast<uint4*>(dx + m * C + c) = pack8(f);
  }
}

// ------------------------------------------------------------------------------------------
// AvgPool3d(k, stride 1) over an NDHWC tensor -> fp32 [N][P][ldo] at channel offset coff
// ------------------------------------------------------------------------------------------
// block = (n, output position, 64-channel group); 4 waves split the window, lane = channel
__global__ void avgpool_fwd_kernel(const uint16_t* __restrict__ x, int T, int H, int W, int C, int kt, int kh, int kw,
                                   float* __restrict__ out, int ldo, int coff, int N) {
  const int To = T - kt + 1, Ho = H - kh + 1, Wo = W - kw + 1;
  const int P = To * Ho * Wo;
  const int cg = (C + 63) / 64;
  int b = blockIdx.x;
  const int g = b % cg; b /= cg;
  const int pos = b % P;
  const int n = b / P;
  const int to = pos / (Ho * Wo), ho = (pos / Wo) % Ho, wo = pos % Wo;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = g * 64 + lane;
  const int vol = kt * kh * kw;
  float s = 0.f;
  if (c < C) {
    for (int i = w; i < vol; i += 4) {
      const int a = i / (kh * kw), r = i % (kh * kw), bb = r / kw, d = r % kw;
      s += e2f(x[((((int64_t)n * T + to + a) * H + ho + bb) * W + wo + d) * C + c]);
    }
  }
  __shared__ float red[4][64];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < C) {
    const float t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    out[((int64_t)n * P + pos) * ldo + coff + c] = t / (float)vol;
  }
}

__global__ void avgpool_bwd_kernel(const float* __restrict__ dout, int ldo, int coff, int T, int H, int W, int C,
                                   int kt, int kh, int kw, uint16_t* __restrict__ dx, int N) {
  const int To = T - kt + 1, Ho = H - kh + 1, Wo = W - kw + 1;
  const int64_t total = (int64_t)N * T * H * W * C;
  const float inv = 1.f / (float)(kt * kh * kw);
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    int64_t r = i;
    const int c = r % C; r /= C;
    const int w = r % W; r /= W;
    const int h = r % H; r /= H;
    const int t = r % T; r /= T;
    const int n = (int)r;
    float s = 0.f;
    for (int to = max(0, t - kt + 1); to <= min(To - 1, t); ++to)
      for (int ho = max(0, h - kh + 1); ho <= min(Ho - 1, h); ++ho)
        for (int wo = max(0, w - kw + 1); wo <= min(Wo - 1, w); ++wo)
          s += dout[(((int64_t)n * To + to) * Ho + ho) * Wo * ldo + (int64_t)wo * ldo + coff + c];
    dx[i] = f2e(s * inv);
  }
}

int grid_for(int64_t work) {
  int64_t b = (work + NT - 1) / NT;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

// grid for ROW_VEC_SETUP kernels: ~4 rows per thread-row, capped
int grid_rows(int64_t M, int C) {
  const int rpi = NT / (C / 8);
  int64_t b = (M + (int64_t)rpi * 4 - 1) / ((int64_t)rpi * 4);
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

// tile ranges of the two-level finalize (<= 256: the scratch holds 256 x 2 x C doubles)
int bn_fin_ranges(int tiles) { return std::min(256, std::max(1, (tiles + FIN_TILES_PER_BLOCK - 1) / FIN_TILES_PER_BLOCK)); }

void bn_finalize_launch(const float* part, int tiles, int C, int64_t count, const float* gamma, const float* beta,
                        float* rm, float* rv, int64_t* nbt, float momentum, float eps, float* smean, float* srstd,
                        float* scale, float* shift, hipStream_t s, double* scratch, unsigned* ctr) {
  if (scratch && ctr) {
    hipLaunchKernelGGL(bn_finalize2_kernel, dim3((C + 63) / 64, bn_fin_ranges(tiles)), dim3(NT), 0, s, part, tiles, C,
                       count, gamma, beta, rm, rv, nbt, momentum, eps, smean, srstd, scale, shift, scratch, ctr);
    return;
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(NT), 0, s, part, tiles, C, count, gamma, beta, rm, rv, nbt,
                     momentum, eps, smean, srstd, scale, shift);
}

void bn_eval_affine_launch(int C, const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                           float* scale, float* shift, hipStream_t s) {
  hipLaunchKernelGGL(bn_eval_affine_kernel, dim3((C + 255) / 256), dim3(256), 0, s, C, gamma, beta, rm, rv, eps,
                     scale, shift);
}

void bn_act_launch(const uint16_t* y, int ldy, uint16_t* out, int ldo, const float* scale, const float* shift,
                   int relu, int64_t M, int C, hipStream_t s) {
  hipLaunchKernelGGL(bn_act_kernel, dim3(grid_rows(M, C)), dim3(NT), 0, s, y, ldy, out, ldo, scale, shift, relu,
                     M, C);
}

void res_out_launch(const uint16_t* yc, const float* sc, const float* hc, const uint16_t* y1, const float* s1,
                    const float* h1, const uint16_t* x, int ldx, uint16_t* out, int ldo, uint8_t* mask, int64_t M,
                    int C, hipStream_t s) {
  hipLaunchKernelGGL(res_out_kernel, dim3(grid_rows(M, C)), dim3(NT), 0, s, yc, sc, hc, y1, s1, h1, x, ldx, out,
                     ldo, mask, M, C);
}

int bn_bwd_reduce_blocks(int64_t M, int C, int* rows_per_block) {
  const int vecs = C / 8;
  const int rpi = NT / vecs;
  // aim for ~16 rows per thread-row and at most 2048 blocks
  int64_t rpb = (int64_t)rpi * 16;
  int64_t blocks = (M + rpb - 1) / rpb;
  if (blocks > 2048) { blocks = 2048; rpb = (M + blocks - 1) / blocks; }
  *rows_per_block = (int)rpb;
  return (int)blocks;
}

void bn_bwd_reduce_launch(const uint16_t* g, int ldg, int mask_mode, const void* mo, int ldm, const float* ms,
                          const float* mh, const uint16_t* y0, const float* mean0, const float* rstd0,
                          const uint16_t* y1, const float* mean1, const float* rstd1, int64_t M, int C, int blocks,
                          int rows_per_block, float* part, uint16_t* dzout, int lddz, hipStream_t s) {
  // compile-time mask mode / operand set (as bn_bwd_apply: fewer registers, more waves per SIMD); LDS sized to
  // the reduction slots actually used ([slots][3][C] fp32: 4 wave slots when C/8 < 64, else one per row group),
  // not the 24 KB worst case, so small-C launches are not LDS-occupancy-limited
  const int vecs_ = C / 8;
  const bool wred_ = vecs_ < 64 && (vecs_ & (vecs_ - 1)) == 0;
  const size_t red_lds = (size_t)(wred_ ? NT / 64 : NT / vecs_) * 3 * C * sizeof(float);
#define PVA_RED(MMv, Y0v, Y1v, DZv)                                                                               \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<MMv, Y0v, Y1v, DZv>), dim3(blocks), dim3(NT), red_lds, s, g, ldg, mo, ldm, \
                     ms, mh, y0, mean0, rstd0, y1, mean1, rstd1, M, C, rows_per_block, part, dzout, lddz)
#define PVA_RED_MM(Y0v, Y1v, DZv)                       \
  switch (mask_mode) {                                  \
    case 1: PVA_RED(1, Y0v, Y1v, DZv); break;            \
    case 2: PVA_RED(2, Y0v, Y1v, DZv); break;            \
    case 3: PVA_RED(3, Y0v, Y1v, DZv); break;            \
    default: PVA_RED(0, Y0v, Y1v, DZv); break;           \
  }
  switch ((y0 ? 4 : 0) | (y1 ? 2 : 0) | (dzout ? 1 : 0)) {
    case 0: PVA_RED_MM(false, false, false); break;
    case 1: PVA_RED_MM(false, false, true); break;
    case 2: PVA_RED_MM(false, true, false); break;
    case 3: PVA_RED_MM(false, true, true); break;
    case 4: PVA_RED_MM(true, false, false); break;
    case 5: PVA_RED_MM(true, false, true); break;
    case 6: PVA_RED_MM(true, true, false); break;
    default: PVA_RED_MM(true, true, true); break;
  }
#undef PVA_RED_MM
#undef PVA_RED
}

void bn_bwd_finalize_launch(const float* part, int blocks, int C, int64_t count, int which, const float* gamma,
                            const float* mean, const float* rstd, float* dgamma, float* dbeta, float beta_acc,
                            float* coef, hipStream_t s, double* scratch, unsigned* ctr) {
  if (scratch && ctr) {
    hipLaunchKernelGGL(bn_bwd_finalize2_kernel, dim3((C + 63) / 64, bn_fin_ranges(blocks)), dim3(NT), 0, s, part,
                       blocks, C, count, which, gamma, mean, rstd, dgamma, dbeta, beta_acc, coef, scratch, ctr);
    return;
  }
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(NT), 0, s, part, blocks, C, count, which, gamma, mean, rstd,
                     dgamma, dbeta, beta_acc, coef);
}

void bn_bwd_apply_launch(const uint16_t* g, int ldg, int mask_mode, const void* mo, int ldm, const float* ms,
                         const float* mh, const uint16_t* y0, const float* coef0, uint16_t* dy0, const uint16_t* y1,
                         const float* coef1, uint16_t* dy1, uint16_t* dzout, int lddz, int dz_accum, int64_t M, int C,
                         hipStream_t s) {
  const dim3 grid(grid_rows(M, C)), block(NT);
#define PVA_APPLY(MMv, Y0v, Y1v, DZv)                                                                       \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<MMv, Y0v, Y1v, DZv>), grid, block, 0, s, g, ldg, mo, ldm, ms, mh, y0, \
                     coef0, dy0, y1, coef1, dy1, dzout, lddz, dz_accum, M, C)
#define PVA_APPLY_MM(Y0v, Y1v, DZv)                       \
  switch (mask_mode) {                                    \
    case 1: PVA_APPLY(1, Y0v, Y1v, DZv); break;            \
    case 2: PVA_APPLY(2, Y0v, Y1v, DZv); break;            \
    case 3: PVA_APPLY(3, Y0v, Y1v, DZv); break;            \
    default: PVA_APPLY(0, Y0v, Y1v, DZv); break;           \
  }
  const int sel = (y0 ? 4 : 0) | (y1 ? 2 : 0) | (dzout ? 1 : 0);
  switch (sel) {
    case 1: PVA_APPLY_MM(false, false, true); break;
    case 2: PVA_APPLY_MM(false, true, false); break;
    case 3: PVA_APPLY_MM(false, true, true); break;
    case 4: PVA_APPLY_MM(true, false, false); break;
    case 5: PVA_APPLY_MM(true, false, true); break;
    case 6: PVA_APPLY_MM(true, true, false); break;
    case 7: PVA_APPLY_MM(true, true, true); break;
    default: break;   // nothing to produce
  }
#undef PVA_APPLY_MM
#undef PVA_APPLY
}

void stem_pool_fwd_launch(const uint16_t* y, const float* scale, const float* shift, uint16_t* out, uint8_t* arg,
                          uint16_t* ymax, int NT_, int H, int W, int Ho, int Wo, int C, int ldo, hipStream_t s) {
  hipLaunchKernelGGL(stem_pool_fwd_kernel, dim3(grid_rows((int64_t)NT_ * Ho * Wo, C)), dim3(NT), 0, s, y, scale,
                     shift, out, arg, ymax, NT_, H, W, Ho, Wo, C, ldo);
}

void stem_pool_bn_apply_launch(const uint16_t* dout, int ldd, const uint8_t* arg, const uint16_t* y, const float* ms,
                               const float* mh, const float* coef, uint16_t* dy, int NT_, int H, int W, int Ho, int Wo,
                               int C, hipStream_t s) {
  hipLaunchKernelGGL(stem_pool_bn_apply_kernel, dim3(grid_rows((int64_t)NT_ * Ho * Wo, C)), dim3(NT), 0, s, dout, ldd,
                     arg, y, ms, mh, coef, dy, NT_, H, W, Ho, Wo, C);
}

void stem_pool_bwd_launch(const uint16_t* dout, int ldd, const uint8_t* arg, uint16_t* dact, int NT_, int H, int W,
                          int Ho, int Wo, int C, hipStream_t s) {
  hipLaunchKernelGGL(stem_pool_bwd_kernel, dim3(grid_for((int64_t)NT_ * H * W * (C / 8))), dim3(NT), 0, s, dout, ldd,
                     arg, dact, NT_, H, W, Ho, Wo, C);
}

int avgpool_global_splits(int N, int vol) {
  int S = (1024 + N - 1) / N;            // >= ~1024 blocks over the chip
  if (S > vol / 8) S = vol / 8 > 0 ? vol / 8 : 1;
  return S;
}

void avgpool_fwd_launch(const uint16_t* x, int N, int T, int H, int W, int C, int kt, int kh, int kw, float* out,
                        int ldo, int coff, float* scratch, hipStream_t s) {
  const int P = (T - kt + 1) * (H - kh + 1) * (W - kw + 1);
  if (P == 1 && C % 8 == 0 && C <= 8 * NT && scratch) {   // global pool: split-position partials + final sum
    const int vol = T * H * W;
    const int S = avgpool_global_splits(N, vol);
    hipLaunchKernelGGL(avgpool_global_part_kernel, dim3(N * S), dim3(NT), 0, s, x, vol, C, S, scratch);
    hipLaunchKernelGGL(avgpool_global_final_kernel, dim3((N * C + NT - 1) / NT), dim3(NT), 0, s, scratch, S, C,
                       1.f / (float)vol, out, ldo, coff, N);
    return;
  }
  const int blocks = N * P * ((C + 63) / 64);
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(blocks), dim3(NT), 0, s, x, T, H, W, C, kt, kh, kw, out, ldo, coff, N);
}

void avgpool_bwd_launch(const float* dout, int ldo, int coff, int N, int T, int H, int W, int C, int kt, int kh,
                        int kw, uint16_t* dx, hipStream_t s) {
  const int64_t total = (int64_t)N * T * H * W * C;
  if (kt == T && kh == H && kw == W && C % 8 == 0 && C <= 8 * NT && ldo % 4 == 0 && coff % 4 == 0) {
    const int64_t M = (int64_t)N * T * H * W;
    hipLaunchKernelGGL(avgpool_global_bwd_kernel, dim3(grid_rows(M, C)), dim3(NT), 0, s, dout, ldo, coff, T * H * W, C,
                       1.f / (float)(T * H * W), dx, M);
    return;
  }
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for(total)), dim3(NT), 0, s, dout, ldo, coff, T, H, W, C, kt, kh,
                     kw, dx, N);
}

PVA_NS_END  // namespace PVA_NS
