// Fused backward of the SlowFast lateral connection (fast -> slow conv (7,1,1) / stride (alpha,1,1) / pad 3, BN,
// ReLU, concatenated into the slow pathway): the BN-backward apply and the input gradient
// in ONE pass over the slow-side tensors.
//
//   apply   dy = A*dz + B*y + C            dz = g masked by relu(y*sc + sh) > 0       (bn_bwd_apply, mask mode 2)
//   dgrad   dx[t_in] += sum_{t_out, kt : alpha*t_out + kt - 3 = t_in} dy[t_out] Wkt      (Wkt: [CO][Cf] tap kt)
//
// The unfused path writes dy, then runs the strided temporal dgrad as alpha stride phases, each re-reading all of
// dy (5 reads of it for alpha = 4) next to the read-modify-write of dx.  Here a workgroup owns one clip, 128
// positions of the H x W plane and a 32-channel group of dx, and walks the clip's slow frames once:
//   * dy[t_out] of its positions is formed in registers from g and y (the apply's arithmetic and rounding; dy is
//     also stored when the caller wants it for the weight gradient) and is at once the MFMA B operand (a lane's 8
//     consecutive channels of one position = one 16-B fragment, no transpose);
//   * the seven taps' products Z_kt = dy Wkt^T (A operand: the tap's weight block, pre-arranged in LDS once per
//     workgroup in fragment order from the dgrad pack [Cf][taps][CO], one ds_read_b128 per fragment) land on fast
//     frames alpha*t_out - 3 .. alpha*t_out + 3; taps 0-2 complete the frames the previous slow frame's taps 4-6
//     started (a 3-frame fp32 carry in registers), tap 3 owns its frame alone, taps 4-6 become the next carry:
//     every dx frame is read and written exactly once;
//   * output rows of the 16 x 16 MFMA tiles are permuted (row r of half h = channel 8(r>>2) + 4h + (r&3)) so a lane
//     ends with 8 consecutive channels of one position: 16-B loads of the old dx and 16-B stores;
//   * the old dx of the next slow frame's four output frames is loaded one iteration ahead (and the next g / y),
//     so a wave keeps a whole iteration of loads in flight.
// Accumulation order per output element: fp32 over the channels of each tap, the two taps of a shared frame added in
// fp32, then the old dx, one rounding — the unfused phase GEMM's K-concatenation up to fp32 reassociation.
#include "common.h"

PVA_NS_BEGIN

namespace {

constexpr int LAT_WAVES = 8;
constexpr int LAT_POS = LAT_WAVES * 16;   // positions of a workgroup (one 16-row MFMA tile per wave)
constexpr int LAT_CG = 32;                // dx channels of a workgroup (8 for the stem lateral's 8 fast channels)
constexpr int LAT_KT = 7;
constexpr uint32_t LAT_OOB = 0x80000000u;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t_;

struct LateralBwdParams {
  const uint16_t* g;     // [N*To*HW][ldg] gradient wrt the (post-ReLU) fusion output: a channel slice of the concat
  const uint16_t* y;     // [N*To*HW][CO] fusion conv output (BN input)
  const float* sc;       // BN forward affine (the ReLU mask), [CO]
  const float* sh;
  const float* coef;     // BN backward coefficients [A | B | C] x CO
  const uint16_t* wd;    // dgrad weight pack [Cf][7][CO]
  uint16_t* dy;          // optional [N*To*HW][CO] out: the applied gradient (weight-gradient operand)
  uint16_t* dx;          // [N*Tf*HW][ldx] fast-pathway input gradient, accumulated
  int ldg, ldx, N, To, Tf, HW, Cf, alpha;
};

// CO: slow channels (16: the stem lateral — half a k-step, lanes of k-chunks 2-3 carry zeros); CG: dx channels per
// workgroup, 32 (two 16-row MFMA halves, 8 consecutive channels per lane) or 8 (rows 0-3 of each half: only the
// lanes of k-chunk 0 hold real outputs)
template <int CO, int CG>
__global__ __launch_bounds__(LAT_WAVES * 64) void lateral_bwd_kernel(const LateralBwdParams p) {
  constexpr int KS = CO < 32 ? 1 : CO / 32;      // MFMA k-steps over the slow channels
  constexpr int NFRAG = LAT_KT * 2 * KS;         // weight fragments (tap, half, k-step), 1 KB each
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* cst = reinterpret_cast<float*>(smem + NFRAG * 1024);   // [5][CO]: A B C sc sh
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rho = lane & 15, kc = lane >> 4;
  const int ngrp = p.Cf / CG, ntile = (p.HW + LAT_POS - 1) / LAT_POS;
  const int L = xcd_remap(blockIdx.x, gridDim.x);   // the channel groups of one tile: adjacent ids, one XCD's L2
  const int grp = L % ngrp, rest = L / ngrp;
  const int tile = rest % ntile, n = rest / ntile;
  const int cbase = grp * CG;

  // ---- weight image: fragment f = (kt * 2 + h) * KS + s; lane l's 16 B = W[co = 32 s + 8 (l >> 4) .. + 8][kt][ci],
  //      ci = cbase + 8 (r >> 2) + 4 h + (r & 3) for row r = l & 15 — contiguous in the dgrad pack
  for (int u = tid; u < NFRAG * 64; u += LAT_WAVES * 64) {
    const int l = u & 63, f = u >> 6;
    const int s = f % KS, h = (f / KS) & 1, kt = f / (2 * KS);
    const int r = l & 15;
    const int ci = cbase + 8 * (r >> 2) + 4 * h + (r & 3);
    const int co = 32 * s + 8 * (l >> 4);
    const bool ok = co < CO && 8 * (r >> 2) < CG;
    *reinterpret_cast<uint4*>(smem + (int64_t)u * 16) =
        ok ? *reinterpret_cast<const uint4*>(p.wd + ((int64_t)ci * LAT_KT + kt) * CO + co) : uint4{0, 0, 0, 0};
  }
  for (int i = tid; i < CO; i += LAT_WAVES * 64) {
    cst[i] = p.coef[i];
    cst[CO + i] = p.coef[CO + i];
    cst[2 * CO + i] = p.coef[2 * CO + i];
    cst[3 * CO + i] = p.sc[i];
    cst[4 * CO + i] = p.sh[i];
  }
  __syncthreads();

  // this lane's position (rows past the plane: out-of-range offsets, zero loads, dropped stores)
  const int pos = tile * LAT_POS + wid * 16 + rho;
  const bool live = pos < p.HW;
  const int64_t slow0 = (int64_t)n * p.To * p.HW, fast0 = (int64_t)n * p.Tf * p.HW;
  const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.g + slow0 * p.ldg), (short)0, p.To * p.HW * p.ldg * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.y + slow0 * CO), (short)0, p.To * p.HW * CO * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.dy ? p.dy + slow0 * CO : p.y), (short)0, p.To * p.HW * CO * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.dx + fast0 * p.ldx), (short)0, p.Tf * p.HW * p.ldx * 2, 0x00020000);
  const bool store_dy = p.dy != nullptr && grp == 0;
  const bool kv = 8 * kc < CO;                   // this lane's k-chunk holds slow channels (CO 16: chunks 0-1)
  const bool ov = CG == 32 || kc == 0;           // this lane holds dx outputs
  // slow-side offsets of frame t (lane: its position, channels 32 s + 8 kc ..)
  auto goff = [&](int t, int s) {
    return live && kv ? (uint32_t)(((t * p.HW + pos) * p.ldg + 32 * s + 8 * kc) * 2) : LAT_OOB;
  };
  auto yoff = [&](int t, int s) {
    return live && kv ? (uint32_t)(((t * p.HW + pos) * CO + 32 * s + 8 * kc) * 2) : LAT_OOB;
  };
  // fast-side offset of frame t (lane: its position, 8 channels cbase + 8 kc ..); frames outside the clip: OOB
  auto xoff = [&](int t) {
    return (live && ov && t >= 0 && t < p.Tf) ? (uint32_t)(((t * p.HW + pos) * p.ldx + cbase + 8 * kc) * 2)
                                               : LAT_OOB;
  };

  uint4 G[KS], Y[KS];
  auto load_gy = [&](int t) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      G[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(gr, goff(t, s), 0, 0));
      Y[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yr, yoff(t, s), 0, 0));
    }
  };
  // old dx of the four frames slow frame t completes: alpha t - 3 .. alpha t (taps 0..3)
  auto load_old = [&](int t, uint4 (&o)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, xoff(p.alpha * t - 3 + j), 0, 0));
  };
  auto store_out = [&](int t_in, const uint4& old, const float (&v)[8]) {
    float o[8];
    unpack8(old, o);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += v[e];
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t_, pack8(o)), xr, xoff(t_in), 0, 0);
  };

  float carry[3][8];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) carry[j][e] = 0.f;
  const char* wl = smem + lane * 16;
  // one slow frame: `cur` holds the old dx of its frames, `nxt` receives the next frame's (two named register sets,
  // alternated by the 2x unrolled loop below — no runtime-indexed register array)
  // CO 256: the next frame's g / y (64 VGPRs) are loaded at the top of its own step instead (one spill otherwise)
  constexpr bool PF_GY = KS <= 4;
  auto step = [&](int t, const uint4 (&cur)[4], uint4 (&nxt)[4]) {
    if (!PF_GY) load_gy(t);
    // ---- apply: dy = A * (g masked by relu(y sc + sh)) + B y + C, rounded (bn_bwd_apply's arithmetic)
    ev8_t b[KS];
    // the per-channel constants are re-read from LDS every frame: hoisted out of the loop they pin 5 x 8 x KS VGPRs
    // (measured: 256 VGPRs + spills); the empty asm makes the index opaque to loop-invariant code motion (an index,
    // not the pointer: an opaque pointer loses its LDS address space and the reads become flat loads)
    int z = 0;
    asm volatile("" : "+s"(z));
    const float* cs = cst + z;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int c0 = kv ? 32 * s + 8 * kc : 0;   // (lanes past CO: zero operands, constants of channel 0 unused)
      float dz[8], a[8], o[8];
      unpack8(G[s], dz);
      unpack8(Y[s], a);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dz[e] = (a[e] * cs[3 * CO + c0 + e] + cs[4 * CO + c0 + e]) > 0.f ? dz[e] : 0.f;
        o[e] = cs[c0 + e] * dz[e] + cs[CO + c0 + e] * a[e] + cs[2 * CO + c0 + e];
      }
      const uint4 pk = kv ? pack8(o) : uint4{0, 0, 0, 0};
      if (store_dy) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t_, pk), dyr, yoff(t, s), 0, 0);
      b[s] = __builtin_bit_cast(ev8_t, pk);
    }
    if (t + 1 < p.To) {
      if (PF_GY) load_gy(t + 1);
      load_old(t + 1, nxt);
    }
    // ---- taps: frame alpha t + kt - 3
#pragma unroll
    for (int kt = 0; kt < LAT_KT; ++kt) {
      f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const ev8_t w = *reinterpret_cast<const ev8_t*>(wl + ((kt * 2 + h) * KS + s) * 1024);
          acc[h] = PVA_MFMA16(w, b[s], acc[h], 0, 0, 0);
        }
      float v[8] = {acc[0][0], acc[0][1], acc[0][2], acc[0][3], acc[1][0], acc[1][1], acc[1][2], acc[1][3]};
      if (kt < 3) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += carry[kt][e];
        store_out(p.alpha * t + kt - 3, cur[kt], v);
      } else if (kt == 3) {
        store_out(p.alpha * t, cur[3], v);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) carry[kt - 4][e] = v[e];
      }
    }
  };
  uint4 O0[4], O1[4];
  if (PF_GY) load_gy(0);
  load_old(0, O0);
#pragma unroll 1
  for (int t = 0; t < p.To; t += 2) {
    step(t, O0, O1);
    if (t + 1 < p.To) step(t + 1, O1, O0);
  }
  // frames alpha To - 3 .. alpha To - 1: taps 4-6 of the last slow frame alone
  {
    uint4 o[4];
    load_old(p.To, o);
#pragma unroll
    for (int j = 0; j < 3; ++j) store_out(p.alpha * p.To - 3 + j, o[j], carry[j]);
  }
}

}  // namespace

int lateral_bwd_legal(int CO, int Cf, int alpha, int To, int Tf, int kt, int pad) {
  return ((CO == 16 && Cf == 8) || ((CO == 64 || CO == 128 || CO == 256) && Cf % LAT_CG == 0)) && alpha == 4 && Tf == alpha * To && kt == LAT_KT && pad == 3 &&
         To >= 1;
}

void lateral_bwd_launch(const uint16_t* g, int ldg, const uint16_t* y, const float* sc, const float* sh,
                        const float* coef, const uint16_t* wd, uint16_t* dy, uint16_t* dx, int ldx, int N, int To,
                        int Tf, int HW, int CO, int Cf, int alpha, hipStream_t st) {
  LateralBwdParams p{g, y, sc, sh, coef, wd, dy, dx, ldg, ldx, N, To, Tf, HW, Cf, alpha};
  const int ntile = (HW + LAT_POS - 1) / LAT_POS;
  const int cg = Cf < LAT_CG ? Cf : LAT_CG;
  const dim3 grid(N * ntile * (Cf / cg)), block(LAT_WAVES * 64);
  const size_t lds = (size_t)LAT_KT * 2 * (CO < 32 ? 1 : CO / 32) * 1024 + 5 * CO * 4;
  switch (CO) {
    case 16: hipLaunchKernelGGL((lateral_bwd_kernel<16, 8>), grid, block, lds, st, p); break;
    case 64: hipLaunchKernelGGL((lateral_bwd_kernel<64, 32>), grid, block, lds, st, p); break;
    case 128: hipLaunchKernelGGL((lateral_bwd_kernel<128, 32>), grid, block, lds, st, p); break;
    default: hipLaunchKernelGGL((lateral_bwd_kernel<256, 32>), grid, block, lds, st, p); break;
  }
}

PVA_NS_END  // namespace PVA_NS
