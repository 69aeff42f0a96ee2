// Host/device parameter blocks for the 3-D convolution kernels (NDHWC, bf16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Implicit-GEMM conv used for the forward pass and for dgrad (one kernel, one addressing scheme).
//
// Rows of the GEMM are points q = (b, qt, qh, qw) of a row lattice (Rt, Rh, Rw).  For each spatial dim:
//   output coordinate   o = q * os + or            (where the row is stored; output dims Ot, Oh, Ow)
//   gather base         a = q * as + ao
//   tap j (0 <= j < n)  reads gathered coordinate g = a + dir * j and weight tap d = b0 + j * bs
//   forward : lattice = output grid, os=1 or=0, as=stride ao=-pad, dir=+1, n=k, b0=0 bs=1
//   dgrad   : one launch per stride phase r (input coords i = q*s + r): os=s or=r, as=1,
//             ao=(r + pad - d0)/s, dir=-1, b0=d0 = first tap with d = r + pad (mod s), bs=s,
//             n = ceil((k - d0)/s).  Only contributing taps are visited: no divisibility tests and
//             no MFMA work on structurally-zero operands (stride-2 dgrad does 1/4 of the naive work).
// k is ordered (tap j, channel); the packed weight row has Kfull = taps_full * Cg elements.
struct ConvParams {
  const uint16_t* x;        // gathered tensor (row stride ldx elements)
  const uint16_t* w;        // packed weights [Ngemm][taps_full][Cg]
  uint16_t* y;              // output rows (row stride ldy)
  float* stats;             // optional BN partial sums [m_tiles][2][Ngemm] (forward)
  const float* in_scale;    // optional per-gathered-channel affine (+ReLU) applied on load
  const float* in_shift;
  int affine;               // 0: none, 1: affine, 2: affine + relu
  int accum;                // 1: y += result (read-modify-write, bf16)
  int M, Ngemm, Kfull, Cg;  // rows in this launch, output channels, packed row length, gathered channels
  int ldx, ldy;
  int Gt, Gh, Gw;           // gathered tensor spatial dims
  int Rt, Rh, Rw;           // row lattice dims
  int Ot, Oh, Ow;           // output tensor dims
  int ost, osh, osw, ort, orh, orw;
  int ast, ash, asw, aot, aoh, aow;
  int dir;
  int nt, nh, nw;           // taps visited per dim
  int kh, kw;               // full kernel extents (weight tap index)
  int bt0, bh0, bw0, bts, bhs, bws;
  int check;                // 1: gathered coordinates may leave the tensor (padding) -> bounds tests
  // Optional backward-BN epilogue, used by the dgrad that produces the gradient of a residual-unit
  // output (the next unit's conv_a): v = acc (+ y_old if accum) (+ eres) ; v *= ReLU bit ; store ;
  // per-column partial sums of v, v*xhat0, v*xhat1 for the producing unit's conv_c / branch1 BNs.
  const uint16_t* eres;     // residual gradient rows (row stride ldr), same row mapping as y
  int ldr;
  const uint8_t* emask;     // ReLU mask bits [rows][Ngemm/8]
  const uint16_t* ey0;      // BN inputs [rows][Ngemm] (raw conv outputs)
  const uint16_t* ey1;
  const float* emean0;
  const float* erstd0;
  const float* emean1;
  const float* erstd1;
  float* epart;             // [m_tiles][3][Ngemm] partial (sum v, sum v*xhat0, sum v*xhat1)
  const float* emsc;        // optional ReLU mask from the BN input itself: v *= (y0*emsc + emsh > 0)
  const float* emsh;        //   (mask mode 2: the gradient of a BN whose ReLU output feeds this conv)
  unsigned xbytes, wbytes;  // buffer-resource extents of x and w (uniform-tap loader)
  const float* ebias;       // EPI 1: optional per-column bias added before the ReLU mask
  // Forward residual-unit epilogue (fres = 1; EPI 0): the conv's own BatchNorm is applied from known
  // statistics and the unit output is written directly:
  //   out = relu(acc * fsc + fsh + r)   with r = eres row (identity shortcut) or r = eres * rsc + rsh
  //   (branch1 BN), ReLU bits of the stored bf16 into emask_out [rows][Ngemm/8]; no raw output, no stats.
  int fres;
  const float* fsc;
  const float* fsh;
  const float* rsc;
  const float* rsh;
  uint8_t* emask_out;
  // 1: statistics-only forward (EPI 0 with stats): the per-tile BN partial sums of the bf16-rounded output are
  // produced, the output itself is never stored (exact BN statistics of a folded conv, models/fused.py)
  int nostore;
  // row-lattice decode by magic numbers (m / (Rt*Rh*Rw), r / (Rh*Rw), r / Rw as (umulhi(n, mg) + n) >> sh; exact for
  // 0 <= n < 2^31), filled by conv_igemm_launch: the kernels' integer divisions cost ~35 VALU each, three per row
  unsigned mg_thw, mg_hw, mg_w;
  int sh_thw, sh_hw, sh_w;
};

// Magic-number division helpers (host fills, device divides)
static inline void pva_magic_div(int d, unsigned* m, int* s) {
  int k = 0;
  while ((1LL << k) < d) ++k;
  *s = k;
  *m = (unsigned)((((1ULL << 32) * ((1ULL << k) - (unsigned long long)d)) / (unsigned long long)d + 1) & 0xffffffffULL);
}
__device__ __forceinline__ int pva_fdiv(int n, unsigned m, int s) {
  return (int)((__umulhi((unsigned)n, m) + (unsigned)n) >> s);
}

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
  int slab;                 // 1: deterministic mode — split s stores into partial + s*Cout*K (no atomics)
  unsigned dybytes, xbytes; // buffer-resource extents
  int variant;              // tile variant (0: 16x128, 1: 32x128, 2: 64x64, 3: 128x64, ...); -1 = heuristic
  // Gram mode (BatchNorm folding of a following 1x1 conv): the SAME affine(+relu) is applied to dy too,
  // i.e. partial = act(x)^T act(x); colsum (optional, [splits][Cout]) receives sum_p act(dy)[p][n] from the
  // k-tile-0 blocks of each split
  int dy_affine;
  float* colsum;
  // magic-number decode of a dY position (q / (To*Ho*Wo), q / (Ho*Wo), q / Wo; pva_fdiv), filled by the narrow
  // weight-gradient launcher
  unsigned mg_othw, mg_ohw, mg_wo;
  int sh_othw, sh_ohw, sh_wo;
};
