// Parameter blocks of the fp32 ("--mixed_precision no") kernels (csrc/fp32/*.hip), shared by the kernels and the
// bindings (csrc/runtime/bindings_f32.cpp).  Activations are NDHWC fp32 rows (one row = one (n, t, h, w) position,
// `ld` elements apart), weights fp32.  Convolutions run on MFMA with every fp32 operand split into two bf16 halves
// (hi = bf16(x), lo = bf16(x - hi)) and three products per fragment pair (hi*hi + hi*lo + lo*hi, fp32 accumulation):
// ~16 mantissa bits per operand, at a third of the bf16 MFMA rate — 5x the f32-input MFMA rate on gfx950
// (MI355X_MICROARCH.md, "f32-input MFMA ... runs at the f32 VECTOR rate").
#pragma once
#include <stdint.h>

// Implicit-GEMM convolution C[m][n] = sum_k A[m][k] * B[n][k] (forward, and each stride phase of the input gradient).
//   m: a position of the GEMM grid (Nb, Qt, Qh, Qw); k = (tap j, channel c), c < Cr.
//   A[m][k] = X[nb, qt*st + taps[j].x, qh*sh + taps[j].y, qw*sw + taps[j].z, c]  (0 outside [0,Ti)x[0,Hi)x[0,Wi))
//   B[n][k] = w[n*ldw + taps[j].w*Cr + c]
//   C[m][n] -> y[nb, qt*ost + ort, qh*osh + orh, qw*osw + orw, n]  (+= the old value when accum)
// Optional consumer-side transform of in-range A values: relu?(x*isc[c] + ish[c]).
// Optional BatchNorm statistics of the output: stats[blockIdx.x][0 / 1][n] = sum / sum of squares over the tile's rows.
struct Conv32 {
  const float* x;
  const float* w;
  float* y;
  float* stats;
  const int* taps;  // int4 per tap (dt, dh, dw, weight tap index)
  const float* isc;
  const float* ish;
  int irelu;
  int ldx, ldw, ldy;
  int M, N, K, Cr, accum;
  int Qt, Qh, Qw;
  int Ti, Hi, Wi;
  int st, sh, sw;
  int Yt, Yh, Yw;
  int ost, osh, osw, ort, orh, orw;
};

// Weight gradient dW[n][k] += sum_p dY[p][n] * A[p][k]   (A = the forward gather above over the dY grid, Cr = Cin).
struct Wgrad32 {
  const float* dy;
  const float* x;
  float* dw;
  const int* taps;
  const float* isc;
  const float* ish;
  int irelu;
  int ldd, ldx, ldw;
  int Cout, K, Cin;
  int P;            // positions of the dY grid (Nb*Qt*Qh*Qw)
  int Qt, Qh, Qw;
  int Ti, Hi, Wi;
  int st, sh, sw;
  int chunk;        // positions per workgroup (multiple of 64)
};
