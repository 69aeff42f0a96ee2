// Box-staged weight gradient of stride-1 'same' (1,3,3) convolutions on MFMA (gfx950): the conv_b of every
// slow-pathway bottleneck (64-256 channels).
//
//   dW[co][tap][ci] = sum_p dY[p][co] * act(x)[p + off(tap)][ci]        (act = the producer's BN+ReLU, recomputed)
//
// A workgroup owns a 64 (co) x 64 (ci) block of dW for all 9 taps and walks a range of BOXES (R whole image rows
// of one frame, P = R*W <= 224 positions).  Per box it stages into LDS once:
//   * dY [P positions][64 co] and the input halo [(R+2) x (W+2)][64 ci] through BN+ReLU (padding = 0), both as
//     channel-group planes [8][positions][8 bf16] (the conv_halo.hip image; each plane padded by 64 B so the two
//     16-lane groups of a 32-lane half hit different banks);
// and reduces over the box's positions in 32-position MFMA k-steps, every operand read with the hardware transpose
// read ds_read_b64_tr_b16 (each lane supplies its own row = position address, so the tap shift and the box's row
// wrap are per-lane offsets into the same halo image — no im2col, no re-read of a tap from L2).
//   * 4 waves, wave w = input channels 16w..16w+15 x all 9 taps x all 64 output channels: 36 accumulators of
//     16x16 (144 VGPRs), kept in registers across every box of the workgroup; per k-step 8 dY + 18 halo
//     transposed reads feed 36 MFMAs (~370 B of LDS per MFMA).
//   * MFMA operands swapped (D = act(x)^T dY) so a lane holds 4 consecutive input channels of one output
//     channel: the workgroup's dW block leaves as 16-B stores into its own slab [split][Cout][9*Cin] (no
//     atomics), summed in a fixed order by wgrad_box_reduce (bitwise-reproducible weight gradients).
// Launch: grid = (Cout/64)*(Cin/64) groups x p.splits box ranges of p.p_per_split boxes (the groups of one range are
// XCD neighbours, so a box's dY / halo slices are re-read from that XCD's L2).
#include "common.h"
#include "conv_params.h"

PVA_NS_BEGIN

namespace {

constexpr int WB_THREADS = 256;
constexpr int WB_PMAX = 224;

__host__ __device__ inline int wb_rows(int H, int W) {
  for (int r = H; r >= 1; --r)
    if (H % r == 0 && r * W <= WB_PMAX) return r;
  return 0;
}

__device__ __forceinline__ s16x4_t tr_read(const char* base) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(base));
}

__device__ __forceinline__ ev8_t cat8(s16x4_t a, s16x4_t b) {
  const s16x8_t v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(ev8_t, v);
}

template <int AFF>
__global__ __launch_bounds__(WB_THREADS, 2) void wgrad_box_kernel(const WgradParams p, const int R) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int W = p.Wo, H = p.Ho;
  const int PW = W + 2;
  const int P = R * W;
  const int PP = (P + 31) & ~31;
  const int NPOS = (R + 2) * PW;
  const int NPOSP = (NPOS + 15) & ~15;
  const int APL = PP * 16 + 64, BPL = NPOSP * 16 + 64;
  char* Aimg = smem;                                        // [8][PP][8] dY
  char* Bimg = smem + 8 * APL;                              // [8][NPOSP][8] act(x) halo
  int* bpos = reinterpret_cast<int*>(Bimg + 8 * BPL);       // [PP] halo position of each box position
  float* aff = reinterpret_cast<float*>(bpos + PP);          // [2][64]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ngi = p.Cin / 64;
  const int groups = (p.Cout / 64) * ngi;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lid / groups, grp = lid - (lid / groups) * groups;
  const int co0 = (grp / ngi) * 64, ci0 = (grp - (grp / ngi) * ngi) * 64;
  const int tpf = H / R;
  const int nboxes = p.P / P;
  const int b_begin = split * p.p_per_split, b_end = min(nboxes, b_begin + p.p_per_split);

  for (int k = tid; k < PP; k += WB_THREADS) {
    // MFMA pad positions (k >= P, dY rows of zeros) point at the first interior halo position, so that every tap
    // offset of theirs stays inside the halo image: reading outside it (uninitialised LDS) could give 0 * NaN
    int v = PW + 1;
    if (k < P) {
      const int h = k / W, w = k - h * W;
      v = (h + 1) * PW + (w + 1);
    }
    bpos[k] = v;
  }
  if constexpr (AFF != 0) {
    for (int i = tid; i < 64; i += WB_THREADS) { aff[i] = p.in_scale[ci0 + i]; aff[64 + i] = p.in_shift[ci0 + i]; }
  }
  for (int idx = tid; idx < 8 * (PP - P); idx += WB_THREADS) {   // dY pad positions stay zero for every box
    const int cg = idx / (PP - P), k = P + (idx - cg * (PP - P));
    *reinterpret_cast<uint4*>(Aimg + cg * APL + k * 16) = uint4{0, 0, 0, 0};
  }

  // transposed-read roles: 16-lane group g, row q of the 4-row block, column quad pq (channels 4pq..4pq+3)
  const int g = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3;
  const int offA = (pq >> 1) * APL + (pq & 1) * 8;                 // + 2*cb*APL + position*16
  const int offB = (2 * wid + (pq >> 1)) * BPL + (pq & 1) * 8;     // + halo position*16
  int toff[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int jh = t / 3, jw = t - jh * 3;
    toff[t] = ((jh - p.ph) * PW + (jw - p.pw)) * 16;
  }

  f32x4_t acc[4][9];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[c][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // staging roles: channel group cg, positions (tid >> 6) * 8 + (tid & 7) + 32 * pass
  const int scg = (tid >> 3) & 7;
  const int sb0 = (tid >> 6) * 8 + (tid & 7);
  float sc[8], sh[8];
  if constexpr (AFF != 0) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) { sc[e] = aff[scg * 8 + e]; sh[e] = aff[64 + scg * 8 + e]; }
  }

  for (int b = b_begin; b < b_end; ++b) {
    const int frame = b / tpf, r0 = (b - frame * tpf) * R;
    const int fbase = frame * H * W;
    __syncthreads();   // previous box fully consumed (and the tables above written)
    // ---- dY rows fbase + r0*W + k
    {
      const uint16_t* src = p.dy + (size_t)(fbase + r0 * W) * p.ldd + co0 + scg * 8;
      constexpr int BATCH = 4;
      for (int k0 = sb0; k0 < P; k0 += 32 * BATCH) {
        uint4 v[BATCH];
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
          const int k = k0 + 32 * u;
          v[u] = k < P ? *reinterpret_cast<const uint4*>(src + (size_t)k * p.ldd) : uint4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
          const int k = k0 + 32 * u;
          if (k < P) *reinterpret_cast<uint4*>(Aimg + scg * APL + k * 16) = v[u];
        }
      }
    }
    // ---- input halo through BN+ReLU (padding positions are zeros of the activation)
    {
      int hh = sb0 / PW, ww = sb0 - (sb0 / PW) * PW;
      constexpr int BATCH = 4;
      for (int b0 = sb0; b0 < NPOS; b0 += 32 * BATCH) {
        uint4 v[BATCH];
        bool ok[BATCH];
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
          const int h = r0 - 1 + hh, w = ww - 1;
          ok[u] = b0 + 32 * u < NPOS && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
          v[u] = ok[u] ? *reinterpret_cast<const uint4*>(p.x + (size_t)(fbase + h * W + w) * p.ldx + ci0 + scg * 8)
                       : uint4{0, 0, 0, 0};
          ww += 32;
          while (ww >= PW) { ww -= PW; ++hh; }
        }
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
          const int bb = b0 + 32 * u;
          if (bb >= NPOS) break;
          uint4 o = v[u];
          if constexpr (AFF != 0) {
            float f[8];
            unpack8(o, f);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = __builtin_fmaf(f[e], sc[e], sh[e]);
            o = pack8_fast(f);
            if constexpr (AFF == 2) o = relu_e16x8(o);
            if (!ok[u]) o = uint4{0, 0, 0, 0};
          }
          *reinterpret_cast<uint4*>(Bimg + scg * BPL + bb * 16) = o;
        }
      }
    }
    __syncthreads();
    // ---- 32-position k-steps
    for (int kc = 0; kc < PP; kc += 32) {
      const int k0 = kc + 8 * g + q;
      ev8_t af[4];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        af[c] = cat8(tr_read(Aimg + offA + 2 * c * APL + k0 * 16), tr_read(Aimg + offA + 2 * c * APL + (k0 + 4) * 16));
      const char* B0 = Bimg + offB + bpos[k0] * 16;
      const char* B1 = Bimg + offB + bpos[k0 + 4] * 16;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const ev8_t xf = cat8(tr_read(B0 + toff[t]), tr_read(B1 + toff[t]));
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c][t] = PVA_MFMA16(xf, af[c], acc[c][t], 0, 0, 0);
      }
    }
  }

  // ---- this workgroup's dW block into its slab: lane holds ci = 16w + 4g + r (r = 0..3) of co = 16c + (lane & 15)
  float* slab = p.partial + (size_t)split * p.Cout * p.K;
  const int col = lane & 15;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int co = co0 + 16 * c + col;
      const int k = t * p.Cin + ci0 + 16 * wid + 4 * g;
      *reinterpret_cast<f32x4_t*>(slab + (size_t)co * p.K + k) = acc[c][t];
    }
}


// ------------------------------------------------------------------------------------------------------------------
// Narrow variant (fast pathway conv_b: Cin = Cout = C in {8, 16, 32}, boxes of P = R*W <= 1024 positions).  dW is tiny
// (C x 9C), so the four waves split the box's 32-position k-steps instead of dW, each keeping the whole 9-tap block
// in registers (9 x ceil(C/16)^2 accumulators) and writing its own slab (slab = 4 * range + wave).  Images are
// position-major [positions][C] (16-64 B per position); the transposed reads of channels >= C (C = 8: column quads
// 2-3 of a 16-wide block) point at a zero block, so the padded MFMA rows / columns are exact zeros.
constexpr int WN_PMAX = 1024;

__host__ __device__ inline int wb_rows_narrow(int H, int W) {
  for (int r = H; r >= 1; --r)
    if (H % r == 0 && r * W <= WN_PMAX) return r;
  return 0;
}

template <int C, int AFF>
__global__ __launch_bounds__(WB_THREADS) void wgrad_box_narrow_kernel(const WgradParams p, const int R) {
  constexpr int NB = (C + 15) / 16;
  constexpr int GP = C / 8;                 // 16-B groups per position
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int W = p.Wo, H = p.Ho;
  const int PW = W + 2;
  const int P = R * W;
  const int PP = (P + 31) & ~31;
  const int NPOS = (R + 2) * PW;
  char* Aimg = smem;                                              // [PP][C] dY
  char* Bimg = Aimg + PP * C * 2;                                 // [NPOS][C] act(x) halo
  char* zero = Bimg + ((NPOS * C * 2 + 15) & ~15);                // 16 zero bytes (+16 pad)
  int* bpos = reinterpret_cast<int*>(zero + 32);                  // [PP]
  float* aff = reinterpret_cast<float*>(bpos + PP);               // [2][C]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int split = xcd_remap(blockIdx.x, gridDim.x);
  const int tpf = H / R;
  const int nboxes = p.P / P;
  const int b_begin = split * p.p_per_split, b_end = min(nboxes, b_begin + p.p_per_split);
  for (int k = tid; k < PP; k += WB_THREADS) {
    // MFMA pad positions (k >= P, dY rows of zeros) point at the first interior halo position, so that every tap
    // offset of theirs stays inside the halo image: reading outside it (uninitialised LDS) could give 0 * NaN
    int v = PW + 1;
    if (k < P) {
      const int h = k / W, w = k - h * W;
      v = (h + 1) * PW + (w + 1);
    }
    bpos[k] = v;
  }
  if (tid < 2) reinterpret_cast<uint4*>(zero)[tid] = uint4{0, 0, 0, 0};
  if constexpr (AFF != 0) {
    for (int i = tid; i < C; i += WB_THREADS) { aff[i] = p.in_scale[i]; aff[C + i] = p.in_shift[i]; }
  }
  for (int idx = tid; idx < (PP - P) * GP; idx += WB_THREADS)
    *reinterpret_cast<uint4*>(Aimg + P * C * 2 + idx * 16) = uint4{0, 0, 0, 0};

  const int g = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3;
  int toff[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int jh = t / 3, jw = t - jh * 3;
    toff[t] = ((jh - p.ph) * PW + (jw - p.pw)) * C * 2;
  }
  // column quad pq of channel block cb: channels 16cb + 4pq .. +3 (>= C -> the zero block, no position stride)
  int cofs[NB];
  bool creal[NB];
#pragma unroll
  for (int cb = 0; cb < NB; ++cb) {
    const int ch = 16 * cb + 4 * pq;
    creal[cb] = ch < C;
    cofs[cb] = ch * 2;
  }
  f32x4_t acc[9][NB][NB];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[t][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int scg = tid % GP;
  float sc[8], sh[8];
  if constexpr (AFF != 0) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) { sc[e] = aff[scg * 8 + e]; sh[e] = aff[C + scg * 8 + e]; }
  }
  constexpr int PPP = WB_THREADS / GP;
  const int sb0 = tid / GP;
  for (int b = b_begin; b < b_end; ++b) {
    const int frame = b / tpf, r0 = (b - frame * tpf) * R;
    const int fbase = frame * H * W;
    __syncthreads();
    {
      const uint16_t* src = p.dy + (size_t)(fbase + r0 * W) * p.ldd + scg * 8;
      constexpr int BATCH = 4;
      for (int k0 = sb0; k0 < P; k0 += PPP * BATCH) {
        uint4 v[BATCH];
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
          const int k = k0 + PPP * u;
          v[u] = k < P ? *reinterpret_cast<const uint4*>(src + (size_t)k * p.ldd) : uint4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
          const int k = k0 + PPP * u;
          if (k < P) *reinterpret_cast<uint4*>(Aimg + k * C * 2 + scg * 16) = v[u];
        }
      }
    }
    {
      int hh = sb0 / PW, ww = sb0 - (sb0 / PW) * PW;
      constexpr int BATCH = 4;
      for (int b0 = sb0; b0 < NPOS; b0 += PPP * BATCH) {
        uint4 v[BATCH];
        bool ok[BATCH];
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
          const int h = r0 - 1 + hh, w = ww - 1;
          ok[u] = b0 + PPP * u < NPOS && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
          v[u] = ok[u] ? *reinterpret_cast<const uint4*>(p.x + (size_t)(fbase + h * W + w) * p.ldx + scg * 8)
                       : uint4{0, 0, 0, 0};
          ww += PPP;
          while (ww >= PW) { ww -= PW; ++hh; }
        }
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
          const int bb = b0 + PPP * u;
          if (bb >= NPOS) break;
          uint4 o = v[u];
          if constexpr (AFF != 0) {
            float f[8];
            unpack8(o, f);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = __builtin_fmaf(f[e], sc[e], sh[e]);
            o = pack8_fast(f);
            if constexpr (AFF == 2) o = relu_e16x8(o);
            if (!ok[u]) o = uint4{0, 0, 0, 0};
          }
          *reinterpret_cast<uint4*>(Bimg + bb * C * 2 + scg * 16) = o;
        }
      }
    }
    __syncthreads();
    for (int kc = wid * 32; kc < PP; kc += 4 * 32) {
      const int k0 = kc + 8 * g + q;
      ev8_t af[NB];
#pragma unroll
      for (int cb = 0; cb < NB; ++cb) {
        const char* a0 = creal[cb] ? Aimg + k0 * C * 2 + cofs[cb] : zero + (pq & 1) * 8;
        const char* a1 = creal[cb] ? Aimg + (k0 + 4) * C * 2 + cofs[cb] : zero + (pq & 1) * 8;
        af[cb] = cat8(tr_read(a0), tr_read(a1));
      }
      const int hb0 = bpos[k0] * C * 2, hb1 = bpos[k0 + 4] * C * 2;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
#pragma unroll
        for (int ci = 0; ci < NB; ++ci) {
          const char* x0 = creal[ci] ? Bimg + hb0 + toff[t] + cofs[ci] : zero + (pq & 1) * 8;
          const char* x1 = creal[ci] ? Bimg + hb1 + toff[t] + cofs[ci] : zero + (pq & 1) * 8;
          const ev8_t xf = cat8(tr_read(x0), tr_read(x1));
#pragma unroll
          for (int co = 0; co < NB; ++co)
            acc[t][ci][co] = PVA_MFMA16(xf, af[co], acc[t][ci][co], 0, 0, 0);
        }
      }
    }
  }
  // this wave's dW into slab 4*range + wave: lane holds ci = 16*cib + 4g + r of co = 16*cob + (lane & 15)
  float* slab = p.partial + (size_t)(split * 4 + wid) * p.Cout * p.K;
  const int col = lane & 15;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int ci = 0; ci < NB; ++ci)
#pragma unroll
      for (int co = 0; co < NB; ++co) {
        const int n = 16 * co + col, c = 16 * ci + 4 * g;
        if (n < C && c < C) *reinterpret_cast<f32x4_t*>(slab + (size_t)n * p.K + t * C + c) = acc[t][ci][co];
      }
}

// Fixed-order slab reduction in two passes: pass 1 sums `per` consecutive slabs per split group (coalesced float4
// over the [Cout][K] block), pass 2 sums the groups and writes grad[co][ci][tap] = beta*grad + scale*v.
__global__ void wgrad_box_sum_kernel(const float* __restrict__ slab, float* __restrict__ tmp, int splits, int per,
                                     int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int g = blockIdx.y;
  const int s0 = g * per, s1 = min(splits, s0 + per);
  const f32x4_t* src = reinterpret_cast<const f32x4_t*>(slab);
  // four slabs in flight per thread (independent accumulators, combined in a fixed order)
  f32x4_t v4[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  int s = s0;
  for (; s + 3 < s1; s += 4) {
    f32x4_t f[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) f[u] = src[(int64_t)(s + u) * n4 + i];
#pragma unroll
    for (int u = 0; u < 4; ++u) v4[u] += f[u];
  }
  for (int u = 0; s < s1; ++s, ++u) v4[u] += src[(int64_t)s * n4 + i];
  reinterpret_cast<f32x4_t*>(tmp)[(int64_t)g * n4 + i] = (v4[0] + v4[1]) + (v4[2] + v4[3]);
}

__global__ void wgrad_box_final_kernel(const float* __restrict__ tmp, int ngroups, int64_t n, float* __restrict__ grad,
                                       int taps, int Cin, int Cin_real, float scale, float beta) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= n) return;
  float v = 0.f;
  for (int gi = 0; gi < ngroups; ++gi) v += tmp[(int64_t)gi * n + a];
  const int per_n = taps * Cin;
  const int co = (int)(a / per_n);
  const int rem = (int)(a - (int64_t)co * per_n);
  const int tap = rem / Cin, c = rem - tap * Cin;
  if (c >= Cin_real) return;
  const int64_t o = ((int64_t)co * Cin_real + c) * taps + tap;
  grad[o] = (beta == 0.f ? 0.f : beta * grad[o]) + scale * v;
}

}  // namespace

// Rows per box when the box-staged kernel can run this weight gradient, else 0 (geometry only; the launch needs
// p.slab-free partial slabs of p.splits * Cout * K floats).
int wgrad_box_legal(const WgradParams& p) {
  if (p.kt != 1 || p.kh != 3 || p.kw != 3 || p.st != 1 || p.sh != 1 || p.sw != 1) return 0;
  if (p.pt != 0 || p.ph != 1 || p.pw != 1) return 0;
  if (p.Ti != p.To || p.Hi != p.Ho || p.Wi != p.Wo) return 0;
  if (p.K != 9 * p.Cin || p.dy_affine || p.ldd % 8 != 0 || p.ldx % 8 != 0) return 0;
  if (p.Cin == p.Cout && (p.Cin == 8 || p.Cin == 16 || p.Cin == 32)) {   // narrow variant
    const int R = wb_rows_narrow(p.Ho, p.Wo);
    return (R > 0 && p.P % (p.Ho * p.Wo) == 0) ? R : 0;
  }
  if (p.Cin % 64 != 0 || p.Cout % 64 != 0) return 0;
  const int R = wb_rows(p.Ho, p.Wo);
  if (R == 0 || p.P % (p.Ho * p.Wo) != 0) return 0;
  return R;
}

template <int C>
void launch_box_narrow(const WgradParams& p, hipStream_t st) {
  const int R = wb_rows_narrow(p.Ho, p.Wo);
  const int W = p.Wo;
  const int PP = (R * W + 31) & ~31;
  const int NPOS = (R + 2) * (W + 2);
  const size_t lds = (size_t)PP * C * 2 + ((size_t)NPOS * C * 2 + 15) / 16 * 16 + 32 + PP * 4 + 2 * C * 4;
  const dim3 grid(p.splits), block(WB_THREADS);
  switch (p.affine) {
    case 0: hipLaunchKernelGGL((wgrad_box_narrow_kernel<C, 0>), grid, block, lds, st, p, R); break;
    case 1: hipLaunchKernelGGL((wgrad_box_narrow_kernel<C, 1>), grid, block, lds, st, p, R); break;
    default: hipLaunchKernelGGL((wgrad_box_narrow_kernel<C, 2>), grid, block, lds, st, p, R); break;
  }
}

void wgrad_box_launch(const WgradParams& p, hipStream_t st) {
  if (p.Cin <= 32) {   // narrow variant: p.splits box ranges, 4 slabs each
    if (p.Cin == 8) launch_box_narrow<8>(p, st);
    else if (p.Cin == 16) launch_box_narrow<16>(p, st);
    else launch_box_narrow<32>(p, st);
    return;
  }
  const int R = wb_rows(p.Ho, p.Wo);
  const int W = p.Wo;
  const int PP = (R * W + 31) & ~31;
  const int NPOSP = (((R + 2) * (W + 2)) + 15) & ~15;
  const size_t lds = (size_t)8 * (PP * 16 + 64) + (size_t)8 * (NPOSP * 16 + 64) + PP * 4 + 2 * 64 * 4;
  const int groups = (p.Cout / 64) * (p.Cin / 64);
  const dim3 grid(groups * p.splits), block(WB_THREADS);
  switch (p.affine) {
    case 0: hipLaunchKernelGGL(wgrad_box_kernel<0>, grid, block, lds, st, p, R); break;
    case 1: hipLaunchKernelGGL(wgrad_box_kernel<1>, grid, block, lds, st, p, R); break;
    default: hipLaunchKernelGGL(wgrad_box_kernel<2>, grid, block, lds, st, p, R); break;
  }
}

// slab [splits][Cout][taps*Cin] -> grad (PyTorch layout [Cout][Cin_real][taps]); tmp holds >= 16 * Cout*taps*Cin
// first-pass groups of the fixed-order slab reduction (the tmp buffer holds this many copies of dW)
int wgrad_box_reduce_groups(int splits) { return splits >= 64 ? 16 : (splits >= 16 ? 4 : 1); }

void wgrad_box_reduce_launch(const float* slab, float* tmp, float* grad, int splits, int Cout, int taps, int Cin,
                             int Cin_real, float scale, float beta, hipStream_t st) {
  const int64_t n = (int64_t)Cout * taps * Cin;
  const int ngroups = wgrad_box_reduce_groups(splits);
  const int per = (splits + ngroups - 1) / ngroups;
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(wgrad_box_sum_kernel, dim3((unsigned)((n4 + 255) / 256), ngroups), dim3(256), 0, st, slab, tmp,
                     splits, per, n4);
  hipLaunchKernelGGL(wgrad_box_final_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, tmp, ngroups, n,
                     grad, taps, Cin, Cin_real, scale, beta);
}

PVA_NS_END  // namespace PVA_NS
