// Weight gradient of gathered (non-1x1 / strided / padded) 3-D convolutions on MFMA (gfx950), split-K over
// positions, with the position -> input-origin decomposition done ONCE per row and shared through LDS.
//
//   dW[n = cout][k = (tap, cin)] = sum_p dY[p][n] * act(im2col(X))[p][k]
//
// Same GEMM mapping, LDS images and hardware-transpose fragment reads (ds_read_b64_tr_b16) as
// conv_wgrad.hip, but built for the issue budget of the compute-bound slow-pathway shapes (3x1x1 temporal
// conv_a of res4/res5, strided branch1, padded (1,3,3) conv_b): the generic kernel re-derives the output
// coordinate of every staged row in every thread that loads a chunk of it (32 threads per row on a
// 256-column tile) with a data-dependent carry loop, which compiled to ~300 VALU + ~150 SALU per 32 MFMAs
// (profiles/r3_wgrad/isa_loops_generic.txt; this kernel: isa_loops_rowtable.txt) — the loop was issue-bound, not MFMA- or memory-bound.
//
// Here one lane per row (wave 0) computes the row's input origin for the stage two steps ahead with
// magic-number divisions (no loops, no divergence) into a 3-deep LDS row table; the loaders read it with
// one ds_read_b128 and do only the tap bounds test + one add per 16-B chunk.  Both operands use raw buffer
// loads (out-of-range -> 0): dY through a resource rebased at the split's first row (rows past the split
// read 0), X through the whole tensor with an out-of-range offset for padding taps.  The producer's
// BN(+ReLU) of X is applied in registers while staging (AFF) and its zero padding re-imposed afterwards.
// One register stage in flight + double-buffered LDS images; BP = 32 or 64 positions per barrier.
// Output: fp32 atomics into one zeroed accumulator, or per-split slabs (deterministic mode).
#pragma once
#include "common.h"
#include "conv_params.h"

PVA_NS_BEGIN

namespace wgrad_rt {

// q / d for 0 <= q < 2^31 with a host-computed magic (Granlund-Montgomery, see magic_div below): 5 VALU, exact.
__device__ __forceinline__ int mdiv(int q, unsigned m, int s1, int s2) {
  const unsigned t = __umulhi((unsigned)q, m);
  return (int)((t + (((unsigned)q - t) >> s1)) >> s2);
}

template <int COLS>
__device__ __forceinline__ int img_off(int row, int colbyte) {
  constexpr int NSEG = COLS * 2 / 32;
  const int seg = colbyte >> 5;
  int h;
  if constexpr (NSEG >= 8) h = (row & 3) | (((row >> 3) & 1) << 2);
  else if constexpr (NSEG == 4) h = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  else if constexpr (NSEG == 2) h = (row >> 3) & 1;
  else h = 0;
  return row * COLS * 2 + (((seg ^ h) << 5) | (colbyte & 31));
}

__device__ __forceinline__ s16x4_t tr_read(const char* base) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(base));
}

// host: m, s1, s2 with q / d == (t + ((q - t) >> s1)) >> s2, t = umulhi(q, m), for every 32-bit q (d >= 1)
inline void magic_div(int d, unsigned* m, int* s1, int* s2) {
  int l = 0;
  while ((1ll << l) < d) ++l;
  *m = (unsigned)(((((unsigned long long)1 << l) - (unsigned long long)d) << 32) / (unsigned long long)d) + 1u;
  *s1 = l < 1 ? l : 1;
  *s2 = l > 1 ? l - 1 : 0;
}

struct RtParams {
  WgradParams p;
  unsigned mWo, mHo, mTo;   // magic divisors of the output dims
  int sWo1, sWo2, sHo1, sHo2, sTo1, sTo2;
};

// AFF: the producer's BN(+ReLU, runtime p.affine == 2) is applied to X on load.  CHECK: taps can leave the
// tensor through padding (bounds test per chunk); otherwise only the end-of-split sentinel is tested.
template <int BMW, int BNW, int WMW, int WNW, int BP, bool AFF, bool CHECK>
__global__ __launch_bounds__((BMW / WMW) * (BNW / WNW) * 64)
void wgrad_rt_kernel(const RtParams rp) {
  const WgradParams& p = rp.p;
  static_assert(BP == 32 || BP == 64, "positions per stage");
  constexpr int NWN = BNW / WNW;
  constexpr int NT = (BMW / WMW) * NWN * 64;
  constexpr int A_CPR = BMW / 8, B_CPR = BNW / 8;
  constexpr int A_CHUNKS = BP * A_CPR, B_CHUNKS = BP * B_CPR;
  constexpr int A_SLOTS = (A_CHUNKS + NT - 1) / NT, B_SLOTS = (B_CHUNKS + NT - 1) / NT;
  constexpr int TM = WMW / 16, TN = WNW / 16;
  constexpr int A_BYTES = BP * BMW * 2, B_BYTES = BP * BNW * 2;
  constexpr int TILE = A_BYTES + B_BYTES;
  constexpr int RT_OFF = 2 * TILE;          // 3-deep row table [3][BP] of int4 after the two image buffers
  static_assert(NT % A_CPR == 0 && NT % B_CPR == 0, "slot mapping");
  static_assert(BP <= 64, "row lanes live in wave 0");
  constexpr unsigned OOB = 0xFFFFFFF0u;   // buffer offset past every extent: the load returns 0
  constexpr int SENT = 0x20000000;          // row past the split: every bounds test fails

  extern __shared__ __attribute__((aligned(16))) char smem[];
  int4* rowtab = reinterpret_cast<int4*>(smem + RT_OFF);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / NWN, wn = wid % NWN;
  const int ntn = (p.Cout + BMW - 1) / BMW, ntk = (p.K + BNW - 1) / BNW;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lid / (ntn * ntk);
  const int tile = lid - split * ntn * ntk;
  const int kt_idx = tile / ntn;
  const int n0 = (tile - kt_idx * ntn) * BMW;
  const int k0 = kt_idx * BNW;
  const int p_begin = split * p.p_per_split;
  const int p_end = min(p.P, p_begin + p.p_per_split);
  const int nsteps = (p_end - p_begin + BP - 1) / BP;

  // dY resource rebased at the split's first row: rows past the split (or P) read as zero
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.dy + (int64_t)p_begin * p.ldd), (short)0, (int)((unsigned)(p_end - p_begin) * (unsigned)p.ldd * 2u),
      0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.xbytes, 0x00020000);

  // ---- A (dY) slots: fixed column, row offset advances by the uniform soffset ----
  const int a_col = tid % A_CPR;
  const int a_n = n0 + a_col * 8;
  unsigned a_vo[A_SLOTS];
  int sa[A_SLOTS];
#pragma unroll
  for (int s = 0; s < A_SLOTS; ++s) {
    const int idx = tid + s * NT;
    const int row = idx / A_CPR;
    // columns past Cout read a real, ignored address (those dW rows are never stored)
    a_vo[s] = (unsigned)(row * p.ldd + (a_n < p.Cout ? a_n : 0)) * 2u;
    sa[s] = img_off<BMW>(row, a_col * 16);
  }

  // ---- B (im2col) slots: fixed (tap, cin) column per thread ----
  const int b_col = tid % B_CPR;
  const int kb = k0 + b_col * 8;
  const bool b_col_ok = kb < p.K;
  int b_dt = 0, b_dh = 0, b_dw = 0, b_c = 0;
  if (b_col_ok) {
    const int tap = kb / p.Cin;
    b_c = kb - tap * p.Cin;
    b_dt = tap / (p.kh * p.kw);
    const int r = tap - b_dt * p.kh * p.kw;
    b_dh = r / p.kw;
    b_dw = r - b_dh * p.kw;
  } else {
    b_dt = SENT;   // column past K: every test fails -> zeros
  }
  const unsigned tapoffb = (unsigned)(((b_dt * p.Hi + b_dh) * p.Wi + b_dw) * p.ldx + b_c) * 2u;
  int b_row[B_SLOTS], sb[B_SLOTS];
#pragma unroll
  for (int s = 0; s < B_SLOTS; ++s) {
    b_row[s] = (tid + s * NT) / B_CPR;
    sb[s] = img_off<BNW>(b_row[s], b_col * 16);
  }
  float asc[8], ash[8];
  if constexpr (AFF) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      asc[e] = b_col_ok ? p.in_scale[b_c + e] : 0.f;
      ash[e] = b_col_ok ? p.in_shift[b_c + e] : 0.f;
    }
  }
  const bool relu = p.affine == 2;

  // ---- row lanes (wave 0, lane r < BP): input origin of row r of stage `st` -> rowtab[st % 3][r] ----
  auto row_info = [&](int st) {
    if (tid < BP) {
      const int q = p_begin + st * BP + tid;
      int4 ri;
      if (st < nsteps && q < p_end) {
        const int hq = mdiv(q, rp.mWo, rp.sWo1, rp.sWo2);
        const int w = q - hq * p.Wo;
        const int tq = mdiv(hq, rp.mHo, rp.sHo1, rp.sHo2);
        const int h = hq - tq * p.Ho;
        const int b = mdiv(tq, rp.mTo, rp.sTo1, rp.sTo2);
        const int t = tq - b * p.To;
        const int bt = t * p.st - p.pt, bh = h * p.sh - p.ph, bw = w * p.sw - p.pw;
        const int bio = (((b * p.Ti + bt) * p.Hi + bh) * p.Wi + bw) * p.ldx;
        ri = make_int4((int)((unsigned)bio * 2u), bt, bh, bw);
      } else {
        ri = make_int4(0, SENT, SENT, SENT);
      }
      rowtab[(st % 3) * BP + tid] = ri;
    }
  };

  uint4 ra[A_SLOTS], rb[B_SLOTS];
  unsigned rb_ok = 0;
  auto load = [&](int st) {
    const unsigned so = (unsigned)(st * BP) * (unsigned)p.ldd * 2u;
#pragma unroll
    for (int s = 0; s < A_SLOTS; ++s)
      ra[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(dyr, (int)a_vo[s], (int)so, 0));
    const int4* rt = rowtab + (st % 3) * BP;
    rb_ok = 0;
#pragma unroll
    for (int s = 0; s < B_SLOTS; ++s) {
      if constexpr (B_CHUNKS % NT != 0) if (tid + s * NT >= B_CHUNKS) break;
      const int4 ri = rt[b_row[s]];
      bool v = (unsigned)(ri.y + b_dt) < (unsigned)p.Ti;
      if constexpr (CHECK) v = v && (unsigned)(ri.z + b_dh) < (unsigned)p.Hi && (unsigned)(ri.w + b_dw) < (unsigned)p.Wi;
      const unsigned off = v ? (unsigned)ri.x + tapoffb : OOB;
      rb[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)off, 0, 0));
      rb_ok |= (v ? 1u : 0u) << s;
    }
  };

  auto store_lds = [&](int buf) {
    char* A = smem + buf * TILE;
    char* B = A + A_BYTES;
#pragma unroll
    for (int s = 0; s < A_SLOTS; ++s) {
      if constexpr (A_CHUNKS % NT != 0) if (tid + s * NT >= A_CHUNKS) break;
      *reinterpret_cast<uint4*>(A + sa[s]) = ra[s];
    }
#pragma unroll
    for (int s = 0; s < B_SLOTS; ++s) {
      if constexpr (B_CHUNKS % NT != 0) if (tid + s * NT >= B_CHUNKS) break;
      uint4 v = rb[s];
      if constexpr (AFF) {
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = __builtin_fmaf(f[e], asc[e], ash[e]);
        v = pack8_fast(f);
        if (relu) v = relu_e16x8(v);
        if (!((rb_ok >> s) & 1u)) v = uint4{0, 0, 0, 0};   // padding / past-the-split rows stay zero
      }
      *reinterpret_cast<uint4*>(B + sb[s]) = v;
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // prologue: row tables of stages 0..2, stage 0 staged, stage 1 in registers
  row_info(0);
  row_info(1);
  row_info(2);
  __syncthreads();
  if (nsteps > 0) {
    load(0);
    store_lds(0);
  }
  if (nsteps > 1) load(1);

  const int g = lane >> 4, li = lane & 15;
  const int tr_row = 8 * g + (li >> 2);
  const int tr_colb = (li & 3) * 8;
  int ta[TM][2], tb[TN][2];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int cb = (wm * WMW + i * 16) * 2 + tr_colb;
    ta[i][0] = img_off<BMW>(tr_row, cb);
    ta[i][1] = img_off<BMW>(tr_row + 4, cb);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cb = (wn * WNW + j * 16) * 2 + tr_colb;
    tb[j][0] = A_BYTES + img_off<BNW>(tr_row, cb);
    tb[j][1] = A_BYTES + img_off<BNW>(tr_row + 4, cb);
  }

  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    // stage `step` is visible in LDS[cur]; every wave is done reading LDS[cur ^ 1] (stage step - 1).  The
    // row-table slot row_info(step + 3) overwrites is stage step's, last read by load(step) two barriers ago
    __syncthreads();
    if (step + 1 < nsteps) {
      store_lds(cur ^ 1);
      if (step + 2 < nsteps) load(step + 2);
    }
    row_info(step + 3);
    const char* A = smem + cur * TILE;
#pragma unroll
    for (int kk = 0; kk < BP / 32; ++kk) {
      ev8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        s16x4_t lo = tr_read(A + kk * 32 * BMW * 2 + ta[i][0]);
        s16x4_t hi = tr_read(A + kk * 32 * BMW * 2 + ta[i][1]);
        s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(ev8_t, v);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        s16x4_t lo = tr_read(A + kk * 32 * BNW * 2 + tb[j][0]);
        s16x4_t hi = tr_read(A + kk * 32 * BNW * 2 + tb[j][1]);
        s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(ev8_t, v);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = PVA_MFMA16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  // D[n][k]: lane holds k = col (lane & 15), n = 4 (lane >> 4) + r
  float* out = p.partial + (p.slab ? (int64_t)split * p.Cout * p.K : 0);
  const bool atomic = p.splits > 1 && !p.slab;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int k = k0 + wn * WNW + j * 16 + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wm * WMW + i * 16 + 4 * g + r;
        if (n < p.Cout && k < p.K) {
          if (atomic) atomicAdd(out + (int64_t)n * p.K + k, acc[i][j][r]);
          else out[(int64_t)n * p.K + k] = acc[i][j][r];
        }
      }
    }
}

template <int BMW, int BNW, int WMW, int WNW, int BP, bool AFF, bool CHECK>
void launch(const RtParams& rp, hipStream_t stream) {
  const WgradParams& p = rp.p;
  constexpr int NT = (BMW / WMW) * (BNW / WNW) * 64;
  const dim3 grid(((p.Cout + BMW - 1) / BMW) * ((p.K + BNW - 1) / BNW) * p.splits);
  const size_t lds = 2 * BP * (BMW + BNW) * 2 + 3 * BP * 16;
  hipLaunchKernelGGL((wgrad_rt_kernel<BMW, BNW, WMW, WNW, BP, AFF, CHECK>), grid, dim3(NT), lds, stream, rp);
}

// tile index (as conv_wgrad_tile): 2: 64x64, 3: 128x64, 4: 128x128, 5: 256x128, 6: 128x256, 7: 256x256
template <int BP, bool AFF, bool CHECK>
void launch_tile(int v, const RtParams& rp, hipStream_t stream) {
  switch (v) {
    case 2: launch<64, 64, 32, 32, BP, AFF, CHECK>(rp, stream); break;
    case 3: launch<128, 64, 64, 32, BP, AFF, CHECK>(rp, stream); break;
    case 4: launch<128, 128, 64, 64, BP, AFF, CHECK>(rp, stream); break;
    case 5: launch<256, 128, 64, 64, BP, AFF, CHECK>(rp, stream); break;
    case 6: launch<128, 256, 64, 64, BP, AFF, CHECK>(rp, stream); break;
    default: launch<256, 256, 128, 64, BP, AFF, CHECK>(rp, stream); break;
  }
}

template <bool AFF>
void launch_aff(int v, bool bp64, bool check, const RtParams& rp, hipStream_t stream) {
  if (bp64) {
    if (check) launch_tile<64, AFF, true>(v, rp, stream); else launch_tile<64, AFF, false>(v, rp, stream);
  } else {
    if (check) launch_tile<32, AFF, true>(v, rp, stream); else launch_tile<32, AFF, false>(v, rp, stream);
  }
}

}  // namespace wgrad_rt

PVA_NS_END  // namespace PVA_NS
