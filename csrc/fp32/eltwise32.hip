// fp32 BatchNorm / activation / pooling / layout kernels of the "--mixed_precision no" path (NDHWC rows).
//
// Row kernels share one layout: a 256-thread block is (QCt channel quads) x (RL row lanes); each thread owns 4
// consecutive channels (float4) and walks rows RL apart, so every wave-load is contiguous along channels and no
// per-element division is needed.  BatchNorm statistics are two-level: per-block fp32 partial sums [R][2][C], then one
// finalize that sums the partials in double (bn32_finalize), also used for the backward reductions.
#include "../kernels/common.h"

namespace pva_f32 {

struct RowMap {
  int QC, QCt, RL, q, rl;
  __device__ RowMap(int C) {
    QC = C >> 2;
    QCt = QC < 256 ? QC : 256;
    RL = 256 / QCt;
    q = threadIdx.x % QCt;
    rl = threadIdx.x / QCt;
  }
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, const float4& v) { *reinterpret_cast<float4*>(p) = v; }

// mode 0: s1 = sum y, s2 = sum y^2.  mode 1: g = relu ? (o > 0 ? d : 0) : d; s1 = sum g, s2 = sum g*(y - mean).
// Without o (an activation its consumers recompute, models/native32.py) the ReLU mask is fma(y, scale, shift) > 0 with
// scale / shift the forward statistics rows 2 and 3 (``mean`` points at row 0 of that [4][C] table).
// mode 3: column sums only, part[block][C] (second level of the conv epilogue's [tiles][2][N] statistics: C = 2N, so
// the output is again [blocks][2][N]).
__global__ __launch_bounds__(256) void chan_reduce32_kernel(const float* y, int ldy, const float* d, int ldd,
                                                            const float* o, int ldo, const float* mean, int mode,
                                                            int relu, int64_t M, int C, int64_t rpb, float* part) {
  const RowMap rm(C);
  __shared__ float4 red[256][2];
  const int64_t rb = (int64_t)blockIdx.x * rpb, re = min(M, rb + rpb);
  for (int qb = 0; qb < rm.QC; qb += rm.QCt) {
    const int qq = qb + rm.q, c = 4 * qq;
    const bool act = rm.rl < rm.RL && qq < rm.QC;
    float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
    if (act) {
      if (mode == 0 || mode == 3) {
#pragma unroll 4
        for (int64_t r = rb + rm.rl; r < re; r += rm.RL) {
          const float4 v = ld4(y + r * ldy + c);
          s1.x += v.x; s1.y += v.y; s1.z += v.z; s1.w += v.w;
          s2.x = fmaf(v.x, v.x, s2.x); s2.y = fmaf(v.y, v.y, s2.y);
          s2.z = fmaf(v.z, v.z, s2.z); s2.w = fmaf(v.w, v.w, s2.w);
        }
      } else {
        const float4 mu = ld4(mean + c);
        const bool ymask = relu && o == nullptr;
        const float4 sc = ld4(mean + (ymask ? 2 * C : 0) + c), sh = ld4(mean + (ymask ? 3 * C : 0) + c);
#pragma unroll 4
        for (int64_t r = rb + rm.rl; r < re; r += rm.RL) {
          float4 g = ld4(d + r * ldd + c);
          const float4 v = ld4(y + r * ldy + c);
          if (relu) {
            float4 ov;
            if (ymask) ov = make_float4(fmaf(v.x, sc.x, sh.x), fmaf(v.y, sc.y, sh.y), fmaf(v.z, sc.z, sh.z),
                                        fmaf(v.w, sc.w, sh.w));
            else ov = ld4(o + r * ldo + c);
            g.x = ov.x > 0.f ? g.x : 0.f; g.y = ov.y > 0.f ? g.y : 0.f;
            g.z = ov.z > 0.f ? g.z : 0.f; g.w = ov.w > 0.f ? g.w : 0.f;
          }
          s1.x += g.x; s1.y += g.y; s1.z += g.z; s1.w += g.w;
          s2.x = fmaf(g.x, v.x - mu.x, s2.x); s2.y = fmaf(g.y, v.y - mu.y, s2.y);
          s2.z = fmaf(g.z, v.z - mu.z, s2.z); s2.w = fmaf(g.w, v.w - mu.w, s2.w);
        }
      }
    }
    red[threadIdx.x][0] = s1;
    red[threadIdx.x][1] = s2;
    __syncthreads();
    if (rm.rl == 0 && qq < rm.QC) {
      for (int l = 1; l < rm.RL; ++l) {
        const float4 a = red[l * rm.QCt + rm.q][0], b = red[l * rm.QCt + rm.q][1];
        s1.x += a.x; s1.y += a.y; s1.z += a.z; s1.w += a.w;
        s2.x += b.x; s2.y += b.y; s2.z += b.z; s2.w += b.w;
      }
      if (mode == 3) {
        st4(part + (int64_t)blockIdx.x * C + c, s1);
      } else {
        float* pp = part + (int64_t)blockIdx.x * 2 * C;
        st4(pp + c, s1);
        st4(pp + C + c, s2);
      }
    }
    __syncthreads();
  }
}

// Per-channel finalize over R partial rows (double sums).
//   mode 0 (train forward): stat = [mean, rstd, scale, shift]; running mean / unbiased var updated; nbt += 1.
//   mode 1 (backward, fstat = forward stat): dgamma (+)= rstd * s2, dbeta (+)= s1 (gbeta: accumulate factor); coef = [k1, k2, k3] with
//           dy = k1*g + k2*(y - mean) + k3.
//   mode 2 (eval): stat[2..3] = scale / shift from the running statistics (no partials).
__global__ __launch_bounds__(256) void bn32_finalize_kernel(const float* part, int R, int C, int64_t count, int mode,
                                                            const float* gamma, const float* beta, float* rmean,
                                                            float* rvar, int64_t* nbt, float momentum, float eps,
                                                            float* stat, const float* fstat, float* dgamma,
                                                            float* dbeta, float* coef, float gbeta) {
  // 16 channels x 16 row lanes per block: a partial table of R <= 1024 rows is 64 loads deep per lane
  __shared__ double red[16][16][2];
  const int cl = threadIdx.x & 15, l = threadIdx.x >> 4, c = blockIdx.x * 16 + cl;
  double a = 0.0, b = 0.0;
  if (c < C && mode != 2)
    for (int r = l; r < R; r += 16) {
      a += (double)part[(int64_t)r * 2 * C + c];
      b += (double)part[(int64_t)r * 2 * C + C + c];
    }
  red[l][cl][0] = a;
  red[l][cl][1] = b;
  __syncthreads();
  if (l != 0 || c >= C) return;
  for (int i = 1; i < 16; ++i) {
    a += red[i][cl][0];
    b += red[i][cl][1];
  }
  const double n = (double)count;
  const double g = gamma ? (double)gamma[c] : 1.0, bt = beta ? (double)beta[c] : 0.0;
  if (mode == 0) {
    const double mean = a / n;
    double var = b / n - mean * mean;
    var = var > 0.0 ? var : 0.0;
    const double rstd = 1.0 / sqrt(var + (double)eps);
    stat[c] = (float)mean;
    stat[C + c] = (float)rstd;
    stat[2 * C + c] = (float)(g * rstd);
    stat[3 * C + c] = (float)(bt - mean * g * rstd);
    if (rmean != nullptr) {
      rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
      rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * (count > 1 ? var * n / (n - 1.0) : var));
    }
    if (nbt != nullptr && c == 0) nbt[0] += 1;
  } else if (mode == 1) {
    const double rstd = (double)fstat[C + c];
    if (dgamma) dgamma[c] = (float)(b * rstd) + (gbeta != 0.f ? gbeta * dgamma[c] : 0.f);
    if (dbeta) dbeta[c] = (float)a + (gbeta != 0.f ? gbeta * dbeta[c] : 0.f);
    const double k1 = g * rstd;
    coef[c] = (float)k1;
    coef[C + c] = (float)(-k1 * rstd * rstd * b / n);
    coef[2 * C + c] = (float)(-k1 * a / n);
  } else {
    const double rstd = 1.0 / sqrt((double)rvar[c] + (double)eps);
    stat[c] = rmean[c];
    stat[C + c] = (float)rstd;
    stat[2 * C + c] = (float)(g * rstd);
    stat[3 * C + c] = (float)(bt - (double)rmean[c] * g * rstd);
  }
}

// out = act(y*scale + shift [+ add])
__global__ __launch_bounds__(256) void bn32_apply_kernel(const float* y, int ldy, const float* stat, const float* add,
                                                         int lda, int relu, float* out, int ldo, int64_t M, int C) {
  const RowMap rm(C);
  if (rm.rl >= rm.RL) return;
  for (int qb = 0; qb < rm.QC; qb += rm.QCt) {
    const int qq = qb + rm.q, c = 4 * qq;
    if (qq >= rm.QC) break;
    const float4 s = ld4(stat + 2 * C + c), h = ld4(stat + 3 * C + c);
    for (int64_t r = (int64_t)blockIdx.x * rm.RL + rm.rl; r < M; r += (int64_t)gridDim.x * rm.RL) {
      const float4 v = ld4(y + r * ldy + c);
      float4 o = make_float4(fmaf(v.x, s.x, h.x), fmaf(v.y, s.y, h.y), fmaf(v.z, s.z, h.z), fmaf(v.w, s.w, h.w));
      if (add != nullptr) {
        const float4 a = ld4(add + r * lda + c);
        o.x += a.x; o.y += a.y; o.z += a.z; o.w += a.w;
      }
      if (relu) {
        o.x = fmaxf(o.x, 0.f); o.y = fmaxf(o.y, 0.f); o.z = fmaxf(o.z, 0.f); o.w = fmaxf(o.w, 0.f);
      }
      st4(out + r * ldo + c, o);
    }
  }
}

// g = relu ? (o > 0 ? d : 0) : d;  dy = k1*g + k2*(y - mean) + k3;  gout (optional) = g
// (no o: the mask is fma(y, scale, shift) > 0 from the forward statistics fstat [4][C], as in chan_reduce32)
__global__ __launch_bounds__(256) void bn32_bwd_apply_kernel(const float* d, int ldd, const float* o, int ldo,
                                                             int relu, const float* y, int ldy, const float* fstat,
                                                             const float* coef, float* dy, int lddy, float* gout,
                                                             int ldg, int64_t M, int C) {
  const RowMap rm(C);
  if (rm.rl >= rm.RL) return;
  for (int qb = 0; qb < rm.QC; qb += rm.QCt) {
    const int qq = qb + rm.q, c = 4 * qq;
    if (qq >= rm.QC) break;
    const float4 mu = ld4(fstat + c), k1 = ld4(coef + c), k2 = ld4(coef + C + c), k3 = ld4(coef + 2 * C + c);
    const bool ymask = relu && o == nullptr;
    const float4 sc = ld4(fstat + 2 * C + c), sh = ld4(fstat + 3 * C + c);
    for (int64_t r = (int64_t)blockIdx.x * rm.RL + rm.rl; r < M; r += (int64_t)gridDim.x * rm.RL) {
      float4 g = ld4(d + r * ldd + c);
      const float4 v = ld4(y + r * ldy + c);
      if (relu) {
        float4 ov;
        if (ymask) ov = make_float4(fmaf(v.x, sc.x, sh.x), fmaf(v.y, sc.y, sh.y), fmaf(v.z, sc.z, sh.z),
                                    fmaf(v.w, sc.w, sh.w));
        else ov = ld4(o + r * ldo + c);
        g.x = ov.x > 0.f ? g.x : 0.f; g.y = ov.y > 0.f ? g.y : 0.f;
        g.z = ov.z > 0.f ? g.z : 0.f; g.w = ov.w > 0.f ? g.w : 0.f;
      }
      const float4 r4 = make_float4(fmaf(k1.x, g.x, fmaf(k2.x, v.x - mu.x, k3.x)),
                                    fmaf(k1.y, g.y, fmaf(k2.y, v.y - mu.y, k3.y)),
                                    fmaf(k1.z, g.z, fmaf(k2.z, v.z - mu.z, k3.z)),
                                    fmaf(k1.w, g.w, fmaf(k2.w, v.w - mu.w, k3.w)));
      st4(dy + r * lddy + c, r4);
      if (gout != nullptr) st4(gout + r * ldg + c, g);
    }
  }
}

// dst[r*ldd + c] = src[r*lds + c] (+ dst when acc), c < C (channel-slice copies of the lateral concat, gradient sums)
__global__ __launch_bounds__(256) void copy32_kernel(const float* src, int lds, float* dst, int ldd, int64_t M, int C,
                                                     int acc) {
  const RowMap rm(C);
  if (rm.rl >= rm.RL) return;
  for (int qb = 0; qb < rm.QC; qb += rm.QCt) {
    const int qq = qb + rm.q, c = 4 * qq;
    if (qq >= rm.QC) break;
    for (int64_t r = (int64_t)blockIdx.x * rm.RL + rm.rl; r < M; r += (int64_t)gridDim.x * rm.RL) {
      float4 v = ld4(src + r * lds + c);
      if (acc) {
        const float4 o = ld4(dst + r * ldd + c);
        v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
      }
      st4(dst + r * ldd + c, v);
    }
  }
}

// Max pool, window (kt,kh,kw) stride (st,sh,sw) pad (pt,ph,pw), -inf padding, first maximum in scan order.
// out [N][To][Ho][Wo][C]; arg = window index of the maximum (uint8).
__global__ __launch_bounds__(256) void maxpool32_fwd_kernel(const float* x, float* out, uint8_t* arg, int N, int T,
                                                            int H, int W, int To, int Ho, int Wo, int C, int kt,
                                                            int kh, int kw, int st, int sh, int sw, int pt, int ph,
                                                            int pw) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n_out = (int64_t)N * To * Ho * Wo * C;
  if (i >= n_out) return;
  const int c = i % C;
  int64_t t = i / C;
  const int wo = t % Wo; t /= Wo;
  const int ho = t % Ho; t /= Ho;
  const int to = t % To;
  const int n = t / To;
  float best = -INFINITY;
  int bi = 0, idx = 0;
  for (int a = 0; a < kt; ++a)
    for (int b = 0; b < kh; ++b)
      for (int e = 0; e < kw; ++e, ++idx) {
        const int ti = to * st - pt + a, hi = ho * sh - ph + b, wi = wo * sw - pw + e;
        if ((unsigned)ti >= (unsigned)T || (unsigned)hi >= (unsigned)H || (unsigned)wi >= (unsigned)W) continue;
        const float v = x[((((int64_t)n * T + ti) * H + hi) * W + wi) * C + c];
        if (v > best || v != v) {
          best = v;
          bi = idx;
          if (v != v) { a = kt; b = kh; break; }
        }
      }
  out[i] = best;
  arg[i] = (uint8_t)bi;
}

// dx[n,t,h,w,c] = sum of dout over the windows whose maximum was this element (gather, deterministic)
__global__ __launch_bounds__(256) void maxpool32_bwd_kernel(const float* dout, const uint8_t* arg, float* dx, int N,
                                                            int T, int H, int W, int To, int Ho, int Wo, int C, int kt,
                                                            int kh, int kw, int st, int sh, int sw, int pt, int ph,
                                                            int pw) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n_in = (int64_t)N * T * H * W * C;
  if (i >= n_in) return;
  const int c = i % C;
  int64_t t = i / C;
  const int w = t % W; t /= W;
  const int h = t % H; t /= H;
  const int tt = t % T;
  const int n = t / T;
  float s = 0.f;
  // outputs o with o*s - p <= x <= o*s - p + k - 1
  const int t0 = max(0, (tt + pt - kt + st) / st), t1 = min(To - 1, (tt + pt) / st);
  const int h0 = max(0, (h + ph - kh + sh) / sh), h1 = min(Ho - 1, (h + ph) / sh);
  const int w0 = max(0, (w + pw - kw + sw) / sw), w1 = min(Wo - 1, (w + pw) / sw);
  for (int a = t0; a <= t1; ++a)
    for (int b = h0; b <= h1; ++b)
      for (int e = w0; e <= w1; ++e) {
        const int da = tt + pt - a * st, db = h + ph - b * sh, de = w + pw - e * sw;
        if (da < 0 || da >= kt || db < 0 || db >= kh || de < 0 || de >= kw) continue;
        const int64_t o = ((((int64_t)n * To + a) * Ho + b) * Wo + e) * C + c;
        if (arg[o] == (da * kh + db) * kw + de) s += dout[o];
      }
  dx[i] = s;
}

// Stride-1 average pool (head): feat[n][p][coff + c] = mean of x over the window at pooled position p.
__global__ __launch_bounds__(256) void avgpool32_fwd_kernel(const float* x, int N, int T, int H, int W, int C, int kt,
                                                            int kh, int kw, float* feat, int ldf, int coff) {
  const int Pt = T - kt + 1, Ph = H - kh + 1, Pw = W - kw + 1, P = Pt * Ph * Pw;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * P * C) return;
  const int c = i % C;
  const int64_t t = i / C;
  const int pp = t % P, n = t / P;
  const int pw = pp % Pw, ph = (pp / Pw) % Ph, pt = pp / (Pw * Ph);
  double s = 0.0;
  for (int a = 0; a < kt; ++a)
    for (int b = 0; b < kh; ++b)
      for (int e = 0; e < kw; ++e) s += x[((((int64_t)n * T + pt + a) * H + ph + b) * W + pw + e) * C + c];
  feat[((int64_t)n * P + pp) * ldf + coff + c] = (float)(s / (double)(kt * kh * kw));
}

__global__ __launch_bounds__(256) void avgpool32_bwd_kernel(const float* dfeat, int ldf, int coff, int N, int T, int H,
                                                            int W, int C, int kt, int kh, int kw, float* dx) {
  const int Pt = T - kt + 1, Ph = H - kh + 1, Pw = W - kw + 1, P = Pt * Ph * Pw;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * T * H * W * C) return;
  const int c = i % C;
  int64_t t = i / C;
  const int w = t % W; t /= W;
  const int h = t % H; t /= H;
  const int tt = t % T;
  const int n = t / T;
  float s = 0.f;
  for (int a = max(0, tt - kt + 1); a <= min(Pt - 1, tt); ++a)
    for (int b = max(0, h - kh + 1); b <= min(Ph - 1, h); ++b)
      for (int e = max(0, w - kw + 1); e <= min(Pw - 1, w); ++e)
        s += dfeat[((int64_t)n * P + (a * Ph + b) * Pw + e) * ldf + coff + c];
  dx[i] = s / (float)(kt * kh * kw);
}

// x [N][Cin][S] (S = T*H*W) -> y [N][S][Cp], zero channels >= Cin
__global__ __launch_bounds__(256) void to_ndhwc32_kernel(const float* x, float* y, int N, int Cin, int64_t S, int Cp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * S * Cp) return;
  const int c = i % Cp;
  const int64_t t = i / Cp;
  const int64_t s = t % S;
  const int n = t / S;
  y[i] = c < Cin ? x[((int64_t)n * Cin + c) * S + s] : 0.f;
}

// ---------------------------------------------------------------- host launchers
static int row_blocks(int64_t M, int C, int cap) {
  const int QC = C / 4, QCt = QC < 256 ? QC : 256, RL = 256 / QCt;
  int64_t b = (M + RL * 4 - 1) / (RL * 4);
  return (int)(b < 1 ? 1 : b > cap ? cap : b);
}

int chan_reduce32_blocks(int64_t M, int C) { return row_blocks(M, C, 1024); }

void chan_reduce32_launch(const float* y, int ldy, const float* d, int ldd, const float* o, int ldo, const float* mean,
                          int mode, int relu, int64_t M, int C, int blocks, float* part, hipStream_t s) {
  const int64_t rpb = (M + blocks - 1) / blocks;
  hipLaunchKernelGGL(chan_reduce32_kernel, dim3(blocks), dim3(256), 0, s, y, ldy, d, ldd, o, ldo, mean, mode, relu,
                     M, C, rpb, part);
}

void bn32_finalize_launch(const float* part, int R, int C, int64_t count, int mode, const float* gamma,
                          const float* beta, float* rmean, float* rvar, int64_t* nbt, float momentum, float eps,
                          float* stat, const float* fstat, float* dgamma, float* dbeta, float* coef, float gbeta,
                          hipStream_t s) {
  hipLaunchKernelGGL(bn32_finalize_kernel, dim3((C + 15) / 16), dim3(256), 0, s, part, R, C, count, mode, gamma, beta,
                     rmean, rvar, nbt, momentum, eps, stat, fstat, dgamma, dbeta, coef, gbeta);
}

void bn32_apply_launch(const float* y, int ldy, const float* stat, const float* add, int lda, int relu, float* out,
                       int ldo, int64_t M, int C, hipStream_t s) {
  if (M == 0) return;
  hipLaunchKernelGGL(bn32_apply_kernel, dim3(row_blocks(M, C, 8192)), dim3(256), 0, s, y, ldy, stat, add, lda, relu,
                     out, ldo, M, C);
}

void bn32_bwd_apply_launch(const float* d, int ldd, const float* o, int ldo, int relu, const float* y, int ldy,
                           const float* fstat, const float* coef, float* dy, int lddy, float* gout, int ldg, int64_t M,
                           int C, hipStream_t s) {
  if (M == 0) return;
  hipLaunchKernelGGL(bn32_bwd_apply_kernel, dim3(row_blocks(M, C, 8192)), dim3(256), 0, s, d, ldd, o, ldo, relu, y,
                     ldy, fstat, coef, dy, lddy, gout, ldg, M, C);
}

void copy32_launch(const float* src, int lds, float* dst, int ldd, int64_t M, int C, int acc, hipStream_t s) {
  if (M == 0 || C == 0) return;
  hipLaunchKernelGGL(copy32_kernel, dim3(row_blocks(M, C, 8192)), dim3(256), 0, s, src, lds, dst, ldd, M, C, acc);
}

void maxpool32_launch(int bwd, const float* a, float* b, uint8_t* arg, int N, int T, int H, int W, int To, int Ho,
                      int Wo, int C, const int* k, const int* st, const int* pd, hipStream_t s) {
  const int64_t n = bwd ? (int64_t)N * T * H * W * C : (int64_t)N * To * Ho * Wo * C;
  if (n == 0) return;
  const int blocks = (int)((n + 255) / 256);
  if (bwd)
    hipLaunchKernelGGL(maxpool32_bwd_kernel, dim3(blocks), dim3(256), 0, s, a, arg, b, N, T, H, W, To, Ho, Wo, C, k[0],
                       k[1], k[2], st[0], st[1], st[2], pd[0], pd[1], pd[2]);
  else
    hipLaunchKernelGGL(maxpool32_fwd_kernel, dim3(blocks), dim3(256), 0, s, a, b, arg, N, T, H, W, To, Ho, Wo, C, k[0],
                       k[1], k[2], st[0], st[1], st[2], pd[0], pd[1], pd[2]);
}

void avgpool32_launch(int bwd, const float* a, float* b, int N, int T, int H, int W, int C, int kt, int kh, int kw,
                      int ldf, int coff, hipStream_t s) {
  const int P = (T - kt + 1) * (H - kh + 1) * (W - kw + 1);
  const int64_t n = bwd ? (int64_t)N * T * H * W * C : (int64_t)N * P * C;
  if (n == 0) return;
  const int blocks = (int)((n + 255) / 256);
  if (bwd)
    hipLaunchKernelGGL(avgpool32_bwd_kernel, dim3(blocks), dim3(256), 0, s, a, ldf, coff, N, T, H, W, C, kt, kh, kw, b);
  else
    hipLaunchKernelGGL(avgpool32_fwd_kernel, dim3(blocks), dim3(256), 0, s, a, N, T, H, W, C, kt, kh, kw, b, ldf, coff);
}

void to_ndhwc32_launch(const float* x, float* y, int N, int Cin, int64_t S, int Cp, hipStream_t s) {
  const int64_t n = (int64_t)N * S * Cp;
  if (n == 0) return;
  hipLaunchKernelGGL(to_ndhwc32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, y, N, Cin, S, Cp);
}

}  // namespace pva_f32
