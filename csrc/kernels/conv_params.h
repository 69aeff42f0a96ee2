// Host/device parameter blocks for the 3-D convolution kernels (NDHWC, bf16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Implicit-GEMM conv used for the forward pass and for dgrad.
//   forward : rows m = output positions (N,To,Ho,Wo); gathered tensor = X (N,Ti,Hi,Wi,Cin);
//             k = (tap, cin);  B = W  packed [Cout][taps][Cin]
//   dgrad   : rows m = input positions (N,Ti,Hi,Wi);  gathered tensor = dY (N,To,Ho,Wo,Cout);
//             k = (tap, cout); B = Wt packed [Cin][taps][Cout]; valid iff (i + pad - tap) % stride == 0
struct ConvParams {
  const uint16_t* x;        // gathered tensor (row stride ldx elements)
  const uint16_t* w;        // packed weights [Ngemm][K]
  uint16_t* y;              // output rows [M][ldy]
  float* stats;             // optional BN partial sums [m_tiles][2][Ngemm]
  const float* in_scale;    // optional per-gathered-channel affine (+ReLU) applied on load
  const float* in_shift;
  int affine;               // 0: none, 1: affine, 2: affine + relu
  int accum;                // 1: y += result (read-modify-write, bf16)
  int M, Ngemm, K, Cg;      // GEMM dims; Cg = gathered channels (K = taps * Cg)
  int ldx, ldy;
  int Gt, Gh, Gw;           // gathered tensor spatial dims
  int Rt, Rh, Rw;           // row-position spatial dims
  int kt, kh, kw, st, sh, sw, pt, ph, pw;
};

// Weight gradient: dW[n = cout][k = (tap, cin)] = sum_p dY[p][cout] * im2col(X)[p][k]
// Split over p in `splits` slices whose fp32 results are atomically added into one zero-initialised
// accumulator [Cout][K] (plain stores when splits == 1); wgrad_reduce converts it to PyTorch layout.
struct WgradParams {
  const uint16_t* dy;       // [P][ldd]
  const uint16_t* x;        // gathered input activations [N,Ti,Hi,Wi][ldx]
  float* partial;           // [splits][Cout][K]
  const float* in_scale;    // optional affine(+relu) applied to x on load (recompute of BN-ReLU)
  const float* in_shift;
  int affine;
  int P, Cout, K, Cin;
  int ldd, ldx;
  int Ti, Hi, Wi;
  int To, Ho, Wo;
  int kt, kh, kw, st, sh, sw, pt, ph, pw;
  int splits, p_per_split;
};
