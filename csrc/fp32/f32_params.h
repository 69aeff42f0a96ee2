// Parameter blocks of the fp32 ("--mixed_precision no") kernels (csrc/fp32/*.hip), shared by the kernels and the
// bindings (csrc/runtime/bindings_f32.cpp).  Activations are NDHWC fp32 rows (one row = one (n, t, h, w) position,
// `ld` elements apart).  Convolutions run on MFMA with every fp32 operand split into NP bf16 pieces (conv32.hip: NP = 3,
// six products per fragment pair, fp32 accuracy; NP = 2, three products); the implicit GEMM's weights arrive
// pre-split (wpack32: three bf16 planes), activations are split while they are staged.
#pragma once
#include <stdint.h>

// Implicit-GEMM convolution C[m][n] = sum_k A[m][k] * B[n][k] (forward, and each stride phase of the input gradient).
//   m: a position of the GEMM grid (Nb, Qt, Qh, Qw); k = (tap j, channel c), c < Cr.
//   A[m][k] = X[nb, qt*st + taps[j].x, qh*sh + taps[j].y, qw*sw + taps[j].z, c]  (0 outside [0,Ti)x[0,Hi)x[0,Wi))
//   B[n][k] = w[n*ldw + taps[j].w*Cr + c]   (piece q of it at + q * wplane; three bf16 planes)
//   C[m][n] -> y[nb, qt*ost + ort, qh*osh + orh, qw*osw + orw, n]  (+= the old value when accum)
// Optional consumer-side transform of in-range A values: relu?(x*isc[c] + ish[c]).
// Optional BatchNorm statistics of the output: stats[blockIdx.x][0 / 1][n] = sum / sum of squares over the tile's rows.
struct Conv32 {
  const float* x;
  const uint16_t* w;
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
  int wplane;       // elements per weight plane
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
  unsigned mqw, mqh, mqt;   // division by Qw / Qh / Qt as (umulhi(n, m) + n) >> s (set by wgrad32_launch)
  int sqw, sqh, sqt;
};
