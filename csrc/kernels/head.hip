// Classification head of SlowFast / Slow-R50 on gfx950: dropout -> per-position
// Linear -> mean over positions -> softmax cross-entropy, forward AND backward, plus eval argmax /
// correct counts.  Replaces ATen dropout + hipBLASLt + softmax/nll kernels + autograd in the step.
//
// Reference semantics: pytorchvideo create_res_basic_head(pool=None) (reference run.py:109): Dropout(0.5)
// -> Linear over channels-last positions -> AdaptiveAvgPool3d(1); F.cross_entropy mean over the batch
// (run.py:254); eval argmax (run.py:297).  Linear and the position mean commute, so the head is computed as
//   xm[n] = mean_p(drop(feat[n, p]))            (head_pool_kernel)
//   logits = xm W^T + b                          (head_linear_fwd_kernel, f32 MFMA 16x16x4, exact fp32)
//   loss_n = lse(logits[n]) - logits[n, y_n]     (head_ce_kernel; dlogits = (softmax - onehot) * g / N)
//   dW = dlogits^T xm, db = sum_n dlogits        (head_linear_bwd_kernel, f32 MFMA)
//   dfeat[n, p] = (dlogits W)[n] * keep(n,p) * s / P   (head_dfeat_kernel, f32 MFMA)
// Dropout masks come from a counter-based Philox4x32-10 stream keyed by a per-step 64-bit seed, so the
// backward regenerates them instead of storing them (not bitwise torch's stream: documented deviation).
#include "common.h"

PVA_NS_BEGIN

namespace {

// ---------------------------------------------------------------------------------- Philox4x32-10
__device__ __forceinline__ uint4 philox(uint32_t k0, uint32_t k1, uint4 c) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
    const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    c = make_uint4(h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// keep-mask of element i (flat index into [N][P][C]): uniform 24-bit draw >= p
__device__ __forceinline__ bool keep_elem(uint32_t k0, uint32_t k1, uint64_t i, uint32_t thresh24) {
  const uint4 r = philox(k0, k1, make_uint4((uint32_t)(i >> 2), (uint32_t)(i >> 34), 0x5eedu, 0u));
  const uint32_t w = (i & 3) == 0 ? r.x : (i & 3) == 1 ? r.y : (i & 3) == 2 ? r.z : r.w;
  return (w >> 8) >= thresh24;
}

typedef __attribute__((ext_vector_type(4))) float f4;

// xm[n][c] = scale/P * sum_p keep * feat[n][p][c]   (thresh24 = 0: no dropout)
__global__ void head_pool_kernel(const float* __restrict__ feat, int N, int P, int C, float* __restrict__ xm,
                                 uint32_t k0, uint32_t k1, uint32_t thresh24, float keep_scale,
                                 const uint64_t* __restrict__ seedp) {
  if (seedp) { const uint64_t sd = *seedp; k0 = (uint32_t)sd; k1 = (uint32_t)(sd >> 32); }
  const int n = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int p = 0; p < P; ++p) {
    const uint64_t i = ((uint64_t)n * P + p) * C + c;
    const float v = feat[i];
    if (thresh24 == 0 || keep_elem(k0, k1, i, thresh24)) s += v;
  }
  xm[(int64_t)n * C + c] = s * (thresh24 ? keep_scale : 1.f) / (float)P;
}

// one 16x16 output tile per workgroup of 4 waves; the waves split the reduction (interleaved 16-wide
// k-chunks) and combine through LDS.  Lane l loads float4 (k = 4q .. 4q+3, q = l>>4) of row (l&15) of
// both operands and issues 4 MFMAs (element t <-> k = k0 + 4q + t on both sides: a consistent permutation
// of the reduction index).
//   out[i][j] = sum_k A[i][k] * B[j][k]   (A: [Mr][K] row stride lda, B: [Nr][K] row stride ldb)
__device__ __forceinline__ f32x4_t mfma_rows_tile(const float* __restrict__ A, int lda, int Mr,
                                                  const float* __restrict__ B, int ldb, int Nr, int K,
                                                  int i0, int j0, int wave, int lane) {
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  const int r = lane & 15, q = lane >> 4;
  const bool ai = i0 + r < Mr, bj = j0 + r < Nr;
  const float* ap = A + (int64_t)(i0 + r) * lda;
  const float* bp = B + (int64_t)(j0 + r) * ldb;
  const bool vec = (lda % 4) == 0 && (ldb % 4) == 0;   // 16-B aligned rows (uniform per launch)
  for (int k0 = wave * 16; k0 < K; k0 += 64) {
    const int k = k0 + 4 * q;
    f4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
    if (vec && k + 3 < K) {
      if (ai) a = *reinterpret_cast<const f4*>(ap + k);
      if (bj) b = *reinterpret_cast<const f4*>(bp + k);
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (ai && k + t < K) a[t] = ap[k + t];
        if (bj && k + t < K) b[t] = bp[k + t];
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[t], acc, 0, 0, 0);
  }
  return acc;
}

// sum the 4 waves' partial tiles; wave 0 returns the total (D map: col = l&15, row = 4(l>>4)+r)
__device__ __forceinline__ f32x4_t reduce_waves(f32x4_t acc, float* red, int wave, int lane) {
  *reinterpret_cast<f32x4_t*>(red + (wave * 64 + lane) * 4) = acc;
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const f32x4_t o = *reinterpret_cast<const f32x4_t*>(red + (w * 64 + lane) * 4);
      acc += o;
    }
  }
  return acc;
}

// logits[n][k] = sum_c xm[n][c] W[k][c] + b[k]
__global__ __launch_bounds__(256) void head_linear_fwd_kernel(const float* __restrict__ xm, const float* __restrict__ W,
                                                             const float* __restrict__ b, float* __restrict__ logits,
                                                             int N, int K, int C) {
  __shared__ __attribute__((aligned(16))) float red[4 * 64 * 4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i0 = blockIdx.y * 16, j0 = blockIdx.x * 16;
  f32x4_t acc = mfma_rows_tile(xm, C, N, W, C, K, C, i0, j0, wave, lane);
  acc = reduce_waves(acc, red, wave, lane);
  if (wave == 0) {
    const int j = j0 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * (lane >> 4) + r;
      if (i < N && j < K) logits[(int64_t)i * K + j] = acc[r] + (b ? b[j] : 0.f);
    }
  }
}

// per row: loss, argmax, correct flag; training: dlogits = (softmax - onehot) * gscale  (gscale = scale / N)
__global__ __launch_bounds__(256) void head_ce_kernel(const float* __restrict__ logits, const int64_t* __restrict__ labels,
                                                     int K, float gscale, float* __restrict__ dlogits,
                                                     float* __restrict__ row_loss, int* __restrict__ row_correct) {
  const int n = blockIdx.x, t = threadIdx.x;
  const float* x = logits + (int64_t)n * K;
  __shared__ float sv[256];
  __shared__ int si[256];
  float m = -INFINITY;
  int am = 0x7fffffff;
  for (int k = t; k < K; k += 256) {
    const float v = x[k];
    if (v > m || (v == m && k < am)) { m = v; am = k; }
  }
  sv[t] = m; si[t] = am;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {   // max with lowest-index tie break (torch.argmax: first maximum)
    if (t < o) {
      const float a = sv[t], b2 = sv[t + o];
      const int ia = si[t], ib = si[t + o];
      if (b2 > a || (b2 == a && ib < ia)) { sv[t] = b2; si[t] = ib; }
    }
    __syncthreads();
  }
  const float mx = sv[0];
  const int arg = si[0];
  __syncthreads();
  float s = 0.f;
  for (int k = t; k < K; k += 256) s += __expf(x[k] - mx);
  sv[t] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) sv[t] += sv[t + o];
    __syncthreads();
  }
  const float se = sv[0];
  const float lse = mx + __logf(se);
  const int64_t y = labels ? labels[n] : -1;
  if (t == 0) {
    if (row_loss) row_loss[n] = (y >= 0 && y < K) ? lse - x[y] : 0.f;
    if (row_correct) row_correct[n] = (y == (int64_t)arg) ? 1 : 0;
  }
  if (dlogits) {
    const float inv = 1.f / se;
    for (int k = t; k < K; k += 256) {
      const float p = __expf(x[k] - mx) * inv;
      dlogits[(int64_t)n * K + k] = (p - (k == y ? 1.f : 0.f)) * gscale;
    }
  }
}

// loss = sum_n row_loss / N ; counts = {sum correct, N}  (one block, fixed order: deterministic)
__global__ void head_reduce_kernel(const float* __restrict__ row_loss, const int* __restrict__ row_correct, int N,
                                   float* __restrict__ loss, int64_t* __restrict__ counts, int accumulate_counts) {
  __shared__ float sl[256];
  __shared__ int sc[256];
  const int t = threadIdx.x;
  float a = 0.f;
  int c = 0;
  for (int n = t; n < N; n += 256) {
    if (row_loss) a += row_loss[n];
    if (row_correct) c += row_correct[n];
  }
  sl[t] = a; sc[t] = c;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) { sl[t] += sl[t + o]; sc[t] += sc[t + o]; }
    __syncthreads();
  }
  if (t == 0) {
    if (loss) loss[0] = sl[0] / (float)N;
    if (counts) {
      if (accumulate_counts) { counts[0] += sc[0]; counts[1] += N; }
      else { counts[0] = sc[0]; counts[1] = N; }
    }
  }
}

// dW[k][c] (+)= sum_n dlogits[n][k] xm[n][c]  via the transposed operands dlT [K][N], xmT [C][N]
// db[k] (+)= sum_n dlogits[n][k]   (blocks with blockIdx.x == 0)
__global__ __launch_bounds__(256) void head_linear_bwd_kernel(const float* __restrict__ dlT, const float* __restrict__ xmT,
                                                             int N, int K, int C, float* __restrict__ dW,
                                                             float* __restrict__ db, float beta) {
  __shared__ __attribute__((aligned(16))) float red[4 * 64 * 4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i0 = blockIdx.y * 16, j0 = blockIdx.x * 16;   // i: output k, j: feature c
  f32x4_t acc = mfma_rows_tile(dlT, N, K, xmT, N, C, N, i0, j0, wave, lane);
  acc = reduce_waves(acc, red, wave, lane);
  if (wave == 0) {
    const int j = j0 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * (lane >> 4) + r;
      if (i < K && j < C) {
        float* d = dW + (int64_t)i * C + j;
        *d = (beta == 0.f ? 0.f : beta * *d) + acc[r];
      }
    }
  }
  if (db && blockIdx.x == 0 && threadIdx.x < 16) {
    const int i = i0 + threadIdx.x;
    if (i < K) {
      float s = 0.f;
      for (int n = 0; n < N; ++n) s += dlT[(int64_t)i * N + n];
      db[i] = (beta == 0.f ? 0.f : beta * db[i]) + s;
    }
  }
}

// [R][Cc] -> [Cc][R] (tiny transposes feeding the MFMA tiles with k-contiguous rows)
__global__ void head_transpose_kernel(const float* __restrict__ in, int R, int Cc, float* __restrict__ out) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 256 threads: 32 x 8
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < R && c < Cc) ? in[(int64_t)r * Cc + c] : 0.f;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int c = c0 + y, r = r0 + tx;
    if (c < Cc && r < R) out[(int64_t)c * R + r] = tile[tx][y];
  }
}

// dfeat[n][p][c] = (sum_k dlogits[n][k] W[k][c]) * keep(n,p,c) * keep_scale / P    via WT [C][K]
__global__ __launch_bounds__(256) void head_dfeat_kernel(const float* __restrict__ dl, const float* __restrict__ WT,
                                                        int N, int K, int C, int P, float* __restrict__ dfeat,
                                                        uint32_t k0, uint32_t k1, uint32_t thresh24, float keep_scale,
                                                        const uint64_t* __restrict__ seedp) {
  if (seedp) { const uint64_t sd = *seedp; k0 = (uint32_t)sd; k1 = (uint32_t)(sd >> 32); }
  __shared__ __attribute__((aligned(16))) float red[4 * 64 * 4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i0 = blockIdx.y * 16, j0 = blockIdx.x * 16;   // i: sample n, j: feature c
  f32x4_t acc = mfma_rows_tile(dl, K, N, WT, K, C, K, i0, j0, wave, lane);
  acc = reduce_waves(acc, red, wave, lane);
  if (wave == 0) {
    const int c = j0 + (lane & 15);
    const float s = (thresh24 ? keep_scale : 1.f) / (float)P;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = i0 + 4 * (lane >> 4) + r;
      if (n < N && c < C) {
        for (int p = 0; p < P; ++p) {
          const uint64_t i = ((uint64_t)n * P + p) * C + c;
          const bool keep = thresh24 == 0 || keep_elem(k0, k1, i, thresh24);
          dfeat[i] = keep ? acc[r] * s : 0.f;
        }
      }
    }
  }
}

// device-resident dropout key (graph-capturable steps: the key advances on the device, one splitmix64 step per
// training forward, instead of being baked into the kernel arguments)
__global__ void head_seed_advance_kernel(uint64_t* __restrict__ s) {
  if (threadIdx.x == 0) {
    uint64_t z = s[0] + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    s[0] = z ^ (z >> 31);
  }
}

__global__ void head_dropout_mask_kernel(int64_t total, uint32_t k0, uint32_t k1, uint32_t thresh24,
                                         uint8_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = keep_elem(k0, k1, (uint64_t)i, thresh24) ? 1 : 0;
}

}  // namespace

static uint32_t thresh_of(float p) {
  if (p <= 0.f) return 0u;
  double t = (double)p * 16777216.0;
  if (t < 1.0) t = 1.0;
  if (t > 16777215.0) t = 16777215.0;
  return (uint32_t)t;
}

// forward of the training/eval head.  feat [N][P][C] fp32; xm scratch [N][C]; logits [N][K].
void head_forward_launch(const float* feat, int N, int P, int C, const float* W, const float* b, int K, float p_drop,
                         uint64_t seed, const uint64_t* seedp, float* xm, float* logits, hipStream_t s) {
  const uint32_t th = thresh_of(p_drop);
  const float ks = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  hipLaunchKernelGGL(head_pool_kernel, dim3((C + 255) / 256, N), dim3(256), 0, s, feat, N, P, C, xm,
                     (uint32_t)seed, (uint32_t)(seed >> 32), th, ks, seedp);
  hipLaunchKernelGGL(head_linear_fwd_kernel, dim3((K + 15) / 16, (N + 15) / 16), dim3(256), 0, s, xm, W, b, logits, N,
                     K, C);
}

// loss / dlogits / counts.  labels int64 [N] (nullable for pure argmax); dlogits nullable (eval).
void head_ce_launch(const float* logits, const int64_t* labels, int N, int K, float gscale, float* dlogits,
                    float* row_loss, int* row_correct, float* loss, int64_t* counts, int acc_counts, hipStream_t s) {
  hipLaunchKernelGGL(head_ce_kernel, dim3(N), dim3(256), 0, s, logits, labels, K, gscale, dlogits, row_loss,
                     row_correct);
  hipLaunchKernelGGL(head_reduce_kernel, dim3(1), dim3(256), 0, s, row_loss, row_correct, N, loss, counts, acc_counts);
}

// backward: dW/db into the flat gradient (beta 0 overwrite / 1 accumulate), dfeat [N][P][C].
// scratch: dlT [K][N], xmT [C][N], WT [C][K]
void head_backward_launch(const float* dlogits, const float* xm, const float* W, int N, int P, int C, int K,
                          float p_drop, uint64_t seed, const uint64_t* seedp, float* dW, float* db, float beta,
                          float* dfeat, float* dlT, float* xmT, float* WT, hipStream_t s) {
  const uint32_t th = thresh_of(p_drop);
  const float ks = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  hipLaunchKernelGGL(head_transpose_kernel, dim3((K + 31) / 32, (N + 31) / 32), dim3(256), 0, s, dlogits, N, K, dlT);
  hipLaunchKernelGGL(head_transpose_kernel, dim3((C + 31) / 32, (N + 31) / 32), dim3(256), 0, s, xm, N, C, xmT);
  hipLaunchKernelGGL(head_transpose_kernel, dim3((C + 31) / 32, (K + 31) / 32), dim3(256), 0, s, W, K, C, WT);
  hipLaunchKernelGGL(head_linear_bwd_kernel, dim3((C + 15) / 16, (K + 15) / 16), dim3(256), 0, s, dlT, xmT, N, K, C,
                     dW, db, beta);
  if (dfeat)
    hipLaunchKernelGGL(head_dfeat_kernel, dim3((C + 15) / 16, (N + 15) / 16), dim3(256), 0, s, dlogits, WT, N, K, C,
                       P, dfeat, (uint32_t)seed, (uint32_t)(seed >> 32), th, ks, seedp);
}

void head_seed_advance_launch(uint64_t* seed, hipStream_t s) {
  hipLaunchKernelGGL(head_seed_advance_kernel, dim3(1), dim3(64), 0, s, seed);
}

void head_dropout_mask_launch(int64_t total, float p_drop, uint64_t seed, uint8_t* out, hipStream_t s) {
  int64_t blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(head_dropout_mask_kernel, dim3((int)blocks), dim3(256), 0, s, total, (uint32_t)seed,
                     (uint32_t)(seed >> 32), thresh_of(p_drop), out);
}

PVA_NS_END  // namespace PVA_NS
