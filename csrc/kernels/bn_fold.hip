// BatchNorm folding for the 1x1 conv_c of a bottleneck unit (gfx950), so its raw output yc is never
// materialised (removes the res_out and BN-apply passes over the widest tensors).
//
// With a = act_b(yb) [M][c] (the conv_c input), Wc [C][c] (bf16 weights as the conv uses them), the Gram
// matrix Ga = a^T a [c][c] and column sums s = 1^T a [c] (both from the wgrad kernel in Gram mode):
//   forward statistics of yc = a Wc^T:  mean_n = (Wc s)_n / M,  E[yc_n^2] = (Wc Ga Wc^T)_nn / M
//   (colsum reduce, T = Wc Ga tiles, per-channel finalize; T is kept for the backward).
// Backward, from dz [M][C] (the ReLU-masked residual gradient), G = dz^T a [C][c] and dbeta = 1^T dz:
//   sum_m dz yc = rowdot(Wc, G),  dgamma = rstd (rowdot - mean dbeta)
//   dyc = A dz + B (yc - mean) + D   with A = g r, B = -g r^2 dgamma / M, D = -g r dbeta / M
//   dWc      = A o G + B o (T - mean s^T) + D s^T                          (bnfold_bwd_grad_kernel)
//   d act_b  = (dz - mean dz) W1 + (a - abar) W2,   W1 = diag(A) Wc,  W2 = Wc^T diag(B) Wc (symmetric):
//              a W2 - abar W2 (1x1 conv + bias) followed by the dgrad of dz with W1 - mean(dz) W1
//              (accumulating, bias epilogue); each mean term uses the bf16 weights of its MFMA so the
//              cancellation happens in fp32 before rounding (bnfold_bias_kernel).
// All reductions are fixed-order (deterministic); the fp32-MFMA tiles use v_mfma_f32_16x16x4_f32.
#include "common.h"

PVA_NS_BEGIN

namespace {

typedef __attribute__((ext_vector_type(4))) float f4;

// 4 consecutive row elements as fp32 from a 16-bit or fp32 row (k multiple of 4, 8-B / 16-B aligned rows)
__device__ __forceinline__ f4 ld4(const uint16_t* row, int k) {
  const uint2 v = *reinterpret_cast<const uint2*>(row + k);
  return f4{lo2f(v.x), hi2f(v.x), lo2f(v.y), hi2f(v.y)};
}
__device__ __forceinline__ f4 ld4(const float* row, int k) { return *reinterpret_cast<const f4*>(row + k); }

// out[i][j] = sum_k A[i][k] * sc[k] * B[j][k]   (16x16 tile; the 4 waves split k in 16-wide chunks)
// rows must be 4-element aligned and K % 4 == 0 (channel counts here are multiples of 8)
template <typename TA, typename TB>
__device__ __forceinline__ f32x4_t tile16(const TA* A, int lda, int Mr, const TB* B, int ldb, int Nr, int K,
                                          const float* sc, int i0, int j0, int wave, int lane) {
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  const int r = lane & 15, q = lane >> 4;
  const bool ai = i0 + r < Mr, bj = j0 + r < Nr;
  const TA* ap = A + (int64_t)(ai ? i0 + r : 0) * lda;
  const TB* bp = B + (int64_t)(bj ? j0 + r : 0) * ldb;
  for (int k0 = wave * 16; k0 < K; k0 += 64) {
    const int k = k0 + 4 * q;
    f4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
    if (k < K) {
      if (ai) a = ld4(ap, k);
      if (bj) b = ld4(bp, k);
      if (sc) a *= ld4(sc, k);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[t], acc, 0, 0, 0);
  }
  return acc;
}

__device__ __forceinline__ f32x4_t reduce4(f32x4_t acc, float* red, int wave, int lane) {
  __syncthreads();
  *reinterpret_cast<f32x4_t*>(red + (wave * 64 + lane) * 4) = acc;
  __syncthreads();
  f32x4_t t = *reinterpret_cast<const f32x4_t*>(red + lane * 4);
#pragma unroll
  for (int w = 1; w < 4; ++w) t += *reinterpret_cast<const f32x4_t*>(red + (w * 64 + lane) * 4);
  return t;   // every wave gets the total
}

// s[j] = sum over the colsum slabs [splits][c]: 16 columns per block, 16 threads per column striding the
// slabs, then a fixed-order 16-way combine (deterministic)
__global__ __launch_bounds__(256) void bnfold_colsum_kernel(const float* __restrict__ sslab, int splits, int c,
                                                            float* __restrict__ s_out) {
  __shared__ float part[16][17];
  const int jl = threadIdx.x & 15, kl = threadIdx.x >> 4;
  const int j = blockIdx.x * 16 + jl;
  float t = 0.f;
  if (j < c) {   // four slab rows in flight per thread, fixed-order combine
    float t4[4] = {0.f, 0.f, 0.f, 0.f};
    int k = kl;
    for (; k + 48 < splits; k += 64) {
      float f[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) f[u] = sslab[(int64_t)(k + 16 * u) * c + j];
#pragma unroll
      for (int u = 0; u < 4; ++u) t4[u] += f[u];
    }
    for (int u = 0; k < splits; k += 16, ++u) t4[u & 3] += sslab[(int64_t)k * c + j];
    t = (t4[0] + t4[1]) + (t4[2] + t4[3]);
  }
  part[kl][jl] = t;
  __syncthreads();
  if (kl == 0 && j < c) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) v += part[q][jl];
    s_out[j] = v;
  }
}

// T = Wc Ga, one 16x16 tile per block (the 4 waves split k), grid (c/16, C/16)
__global__ __launch_bounds__(256) void bnfold_t_kernel(const uint16_t* __restrict__ Wf, const float* __restrict__ Ga,
                                                       int C, int c, float* __restrict__ T) {
  __shared__ __attribute__((aligned(16))) float red[4 * 64 * 4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j0 = blockIdx.x * 16, i0 = blockIdx.y * 16;
  // Ga is symmetric: row j of Ga = column j, so the B operand reads rows (contiguous)
  const f32x4_t t = reduce4(tile16(Wf, c, C, Ga, c, c, c, (const float*)nullptr, i0, j0, wave, lane), red, wave,
                            lane);
  if (wave == 0) {
    const int j = j0 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = i0 + 4 * (lane >> 4) + r;
      if (n < C && j < c) T[(int64_t)n * c + j] = t[r];
    }
  }
}

// one wave per output channel n: mean_n = Wc[n] . s / M, E[yc^2] = Wc[n] . T[n] / M (double accumulation),
// then the training-mode BN finalize (running stats with unbiased variance, consumer affine)
__global__ __launch_bounds__(256) void bnfold_finalize_kernel(
    const uint16_t* __restrict__ Wf, const float* __restrict__ T, const float* __restrict__ s, int C, int c,
    int64_t count, const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ run_mean,
    float* __restrict__ run_var, int64_t* __restrict__ nbt, float momentum, float eps, float* __restrict__ save_mean,
    float* __restrict__ save_rstd, float* __restrict__ scale, float* __restrict__ shift) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= C) return;   // wave-uniform; no barriers below
  double mu = 0.0, q = 0.0;
  for (int j = lane; j < c; j += 64) {
    const double w = (double)e2f(Wf[(int64_t)n * c + j]);
    mu += w * (double)s[j];
    q += w * (double)T[(int64_t)n * c + j];
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    mu += __shfl_xor(mu, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  if (lane == 0) {
    mu /= (double)count;
    double var = q / (double)count - mu * mu;
    if (var < 0) var = 0;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    save_mean[n] = (float)mu;
    save_rstd[n] = rstd;
    const float g = gamma[n], b = beta[n];
    scale[n] = g * rstd;
    shift[n] = b - (float)mu * g * rstd;
    if (run_mean) {
      const double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
      run_mean[n] = (1.f - momentum) * run_mean[n] + momentum * (float)mu;
      run_var[n] = (1.f - momentum) * run_var[n] + momentum * (float)unb;
    }
    if (n == 0 && nbt) nbt[0] += 1;
  }
}

// per output channel n (block): dbeta = sum of the epilogue partials, sdzy = Wc[n] . G[n],
// dgamma = rstd (sdzy - mean dbeta) -> grad buffers (beta-accumulate) and coef [A | B | D] [3][C]
__global__ __launch_bounds__(256) void bnfold_bwd_coef_kernel(
    const float* __restrict__ part, int tiles, const uint16_t* __restrict__ Wf, const float* __restrict__ G, int C,
    int c, int64_t count, const float* __restrict__ gamma, const float* __restrict__ mean,
    const float* __restrict__ rstd, float* __restrict__ dgamma, float* __restrict__ dbeta, float beta_acc,
    float* __restrict__ coef) {
  const int n = blockIdx.x;
  __shared__ double ra[256], rb[256];
  double sdz = 0.0, sy = 0.0;
  {   // four strided partial rows in flight per thread (latency-bound), combined in a fixed order
    double d4[4] = {0.0, 0.0, 0.0, 0.0};
    int t = threadIdx.x;
    for (; t + 768 < tiles; t += 1024) {
      float f[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) f[u] = part[(int64_t)(t + 256 * u) * 3 * C + n];
#pragma unroll
      for (int u = 0; u < 4; ++u) d4[u] += f[u];
    }
    for (int u = 0; t < tiles; t += 256, ++u) d4[u & 3] += part[(int64_t)t * 3 * C + n];
    sdz = (d4[0] + d4[1]) + (d4[2] + d4[3]);
  }
  for (int j = threadIdx.x; j < c; j += 256) sy += (double)e2f(Wf[(int64_t)n * c + j]) * G[(int64_t)n * c + j];
  ra[threadIdx.x] = sdz; rb[threadIdx.x] = sy;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) { ra[threadIdx.x] += ra[threadIdx.x + o]; rb[threadIdx.x] += rb[threadIdx.x + o]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double db = ra[0];
    const double r = rstd[n], mu = mean[n];
    const double dg = r * (rb[0] - mu * db);
    if (dgamma) {
      dgamma[n] = (beta_acc == 0.f ? 0.f : beta_acc * dgamma[n]) + (float)dg;
      dbeta[n] = (beta_acc == 0.f ? 0.f : beta_acc * dbeta[n]) + (float)db;
    }
    const double g = gamma[n], inv = 1.0 / (double)count;
    coef[n] = (float)(g * r);                       // A
    coef[C + n] = (float)(-g * r * r * dg * inv);   // B
    coef[2 * C + n] = (float)(-g * r * db * inv);   // D
    coef[3 * C + n] = (float)(db * inv);            // mean(dz)
  }
}

// elementwise over [C][c]: dWc = A G + B (T - mean s) + D s  -> grad (PyTorch [C][c][1][1][1], beta-accumulate);
// W1t[j][n] = bf16(A_n Wc[n][j])  (the dgrad pack layout [Cin = c][Cout = C]) through a 32x32 LDS transpose
__global__ __launch_bounds__(256) void bnfold_bwd_grad_kernel(
    const float* __restrict__ G, const float* __restrict__ T, const float* __restrict__ s, const float* __restrict__ mean,
    const float* __restrict__ coef, const uint16_t* __restrict__ Wf, int C, int c, float* __restrict__ grad,
    float beta, uint16_t* __restrict__ W1t) {
  __shared__ uint16_t tile[32][33];
  const int j0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8) {
    const int n = n0 + y, j = j0 + tx;
    uint16_t w1 = 0;
    if (n < C && j < c) {
      const int64_t o = (int64_t)n * c + j;
      const float A = coef[n], B = coef[C + n], D = coef[2 * C + n];
      const float v = A * G[o] + B * (T[o] - mean[n] * s[j]) + D * s[j];
      grad[o] = (beta == 0.f ? 0.f : beta * grad[o]) + v;
      w1 = f2e(A * e2f(Wf[o]));
    }
    tile[y][tx] = w1;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int j = j0 + y, n = n0 + tx;
    if (j < c && n < C) W1t[(int64_t)j * C + n] = tile[tx][y];
  }
}

// W2[i][j] = sum_n Wd[i][n] B_n Wd[j][n]  (Wd = the dgrad pack [c][C] = Wc^T) -> bf16 forward pack [c][c];
// grid (c/16, c/16)
__global__ __launch_bounds__(256) void bnfold_w2_kernel(const uint16_t* __restrict__ Wd, const float* __restrict__ coef,
                                                       int C, int c, uint16_t* __restrict__ W2) {
  __shared__ __attribute__((aligned(16))) float red[4 * 64 * 4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i0 = blockIdx.y * 16, j0 = blockIdx.x * 16;
  const f32x4_t t = reduce4(tile16(Wd, C, c, Wd, C, c, C, coef + C, i0, j0, wave, lane), red, wave, lane);
  if (wave == 0) {
    const int j = j0 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * (lane >> 4) + r;
      if (i < c && j < c) W2[(int64_t)i * c + j] = f2e(t[r]);
    }
  }
}

// The two large mean terms of d act_b are cancelled with the SAME bf16-rounded weights the MFMAs use, in fp32
// before any rounding (dz carries the broadcast mean of the pooled-head gradient, which the BN backward
// removes: dz W1 and its mean correction are each far larger than their sum):
//   biasA[j] = -sum_n mean(dz_n) W1b[n][j]   (epilogue of the dz W1 dgrad)
//   biasB[j] = -sum_i abar_i W2b[j][i]       (epilogue of the act_b W2 conv; abar = s / M)
__global__ __launch_bounds__(256) void bnfold_bias_kernel(const uint16_t* __restrict__ W1t,
                                                         const uint16_t* __restrict__ W2b, const float* __restrict__ coef,
                                                         const float* __restrict__ s, int C, int c, int64_t count,
                                                         float* __restrict__ bias) {
  const int j = blockIdx.x;
  __shared__ double r0[256], r1[256];
  double a = 0.0, b = 0.0;
  const double inv = 1.0 / (double)count;
  for (int n = threadIdx.x; n < C; n += 256) a -= (double)coef[3 * C + n] * e2f(W1t[(int64_t)j * C + n]);
  for (int i = threadIdx.x; i < c; i += 256) b -= (double)s[i] * inv * e2f(W2b[(int64_t)j * c + i]);
  r0[threadIdx.x] = a;
  r1[threadIdx.x] = b;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) { r0[threadIdx.x] += r0[threadIdx.x + o]; r1[threadIdx.x] += r1[threadIdx.x + o]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) { bias[j] = (float)r0[0]; bias[c + j] = (float)r1[0]; }
}

}  // namespace

void bnfold_fwd_stats_launch(const uint16_t* Wf, const float* Ga, const float* sslab, int splits, int C, int c,
                             int64_t count, float* T, float* s_out, const float* gamma, const float* beta, float* rm,
                             float* rv, int64_t* nbt, float momentum, float eps, float* smean, float* srstd,
                             float* scale, float* shift, hipStream_t st) {
  hipLaunchKernelGGL(bnfold_colsum_kernel, dim3((c + 15) / 16), dim3(256), 0, st, sslab, splits, c, s_out);
  hipLaunchKernelGGL(bnfold_t_kernel, dim3((c + 15) / 16, (C + 15) / 16), dim3(256), 0, st, Wf, Ga, C, c, T);
  hipLaunchKernelGGL(bnfold_finalize_kernel, dim3((C + 3) / 4), dim3(256), 0, st, Wf, T, s_out, C, c, count, gamma,
                     beta, rm, rv, nbt, momentum, eps, smean, srstd, scale, shift);
}

void bnfold_bwd_launch(const float* part, int tiles, const uint16_t* Wf, const uint16_t* Wd, const float* G,
                       const float* T, const float* s, int C, int c, int64_t count, const float* gamma,
                       const float* mean, const float* rstd, float* dgamma, float* dbeta, float* dW, float beta_acc,
                       float* coef, uint16_t* W1t, uint16_t* W2, float* bias, hipStream_t st) {
  hipLaunchKernelGGL(bnfold_bwd_coef_kernel, dim3(C), dim3(256), 0, st, part, tiles, Wf, G, C, c, count, gamma, mean,
                     rstd, dgamma, dbeta, beta_acc, coef);
  hipLaunchKernelGGL(bnfold_bwd_grad_kernel, dim3((c + 31) / 32, (C + 31) / 32), dim3(256), 0, st, G, T, s, mean, coef,
                     Wf, C, c, dW, beta_acc, W1t);
  hipLaunchKernelGGL(bnfold_w2_kernel, dim3((c + 15) / 16, (c + 15) / 16), dim3(256), 0, st, Wd, coef, C, c, W2);
  hipLaunchKernelGGL(bnfold_bias_kernel, dim3(c), dim3(256), 0, st, W1t, W2, coef, s, C, c, count, bias);
}

PVA_NS_END  // namespace PVA_NS
