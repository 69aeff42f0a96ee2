// Weight gradient of the NDHWC 3-D convolution on MFMA (gfx950), split-K over positions.
//
//   dW[n = cout][k = (tap, cin)] = sum_p dY[p][n] * im2col(X)[p][k]
//
// Both operands are position-major in HBM (channels contiguous), so the reduction axis p is the
// strided one.  Tiles are staged as [p][cols] row-major images (contiguous 16-B loads, the im2col
// side is the same chunk gather as the forward kernel) and the MFMA fragments are read with the gfx950
// hardware-transpose LDS read ds_read_b64_tr_b16 (cdna_hip_programming.md T10): one 16-lane group
// reads a 4(p) x 16(col) block and each lane receives one column's 4 p-values.  32-byte column
// segments are XOR-swizzled with row bits 1 and 3 so the 8 rows a 32-lane half touches land on
// disjoint bank groups.  The p axis is split into slices (XCD-local with their tiles) whose fp32 tiles are added into one
// accumulator with no-return float atomics (≈1.3 TB/s chip-wide; a serial slab reduce was 17 % of the
// step); wgrad_reduce then scatters it into PyTorch's [Cout][Cin][kt][kh][kw] layout, accumulating into
// the fp32 master-gradient buffer, and re-zeroes the accumulator.
#include "common.h"
#include "conv_params.h"
#include "wgrad_rt_impl.h"
#include <type_traits>

PVA_NS_BEGIN

namespace {

// BP (template): positions per LDS stage = 32 (one MFMA k-step) or 64 (two k-steps per barrier pair)

template <int COLS>
__device__ __forceinline__ int img_off(int row, int colbyte) {
  // [BP][COLS] bf16 image of 32-byte segments.  A 32-lane half of a transpose read touches rows
  // {r..r+3, r+8..r+11}; the XOR below gives those 8 rows distinct segments of the 256-byte bank row
  // for every row length (64 B rows: 4 rows share a bank row; 128 B: 2; >= 256 B: 1).
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
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4_t*)(base));
}

// DENSE: 1x1x1, stride 1, no padding — the im2col row of position p is x row p, so both operands stream
// with raw buffer loads whose per-step advance is one SGPR offset (no per-lane address math).
template <int BMW, int BNW, int WMW, int WNW, int CH, int DENSE, int BP>
__global__ __launch_bounds__((BMW / WMW) * (BNW / WNW) * 64)
void conv_wgrad_kernel(const WgradParams p) {
  static_assert(BP == 32 || BP == 64, "positions per stage");
  constexpr int NWN = BNW / WNW;
  constexpr int NT = (BMW / WMW) * NWN * 64;
  constexpr int A_CPR = BMW / 8;            // 16-B chunks per dY row
  constexpr int B_CPR = BNW / CH;           // chunks per im2col row
  constexpr int A_CHUNKS = BP * A_CPR, B_CHUNKS = BP * B_CPR;
  constexpr int A_SLOTS = (A_CHUNKS + NT - 1) / NT;
  constexpr int B_SLOTS = (B_CHUNKS + NT - 1) / NT;
  constexpr int TM = WMW / 16, TN = WNW / 16;
  constexpr int A_BYTES = BP * BMW * 2, B_BYTES = BP * BNW * 2;
  constexpr int TILE = A_BYTES + B_BYTES;
  static_assert(NT % A_CPR == 0 && NT % B_CPR == 0, "slot mapping");
  using VT = typename std::conditional<CH == 8, uint4, uint2>::type;

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / NWN, wn = wid % NWN;
  // 1-D grid, XCD-aware: the (cout, k) tiles of one position split get consecutive logical ids, which the
  // bijective remap keeps on one XCD, so the split's dY / im2col rows are fetched from HBM once and served
  // to the other tiles from that XCD's L2 (the hardware spreads consecutive workgroups over the 8 XCDs)
  const int ntn = (p.Cout + BMW - 1) / BMW, ntk = (p.K + BNW - 1) / BNW;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lid / (ntn * ntk);
  const int tile = lid - split * ntn * ntk;
  const int kt_idx = tile / ntn;
  const int n0 = (tile - kt_idx * ntn) * BMW;   // cout tile
  const int k0 = kt_idx * BNW;                   // k tile
  const int p_begin = split * p.p_per_split;
  const int p_end = min(p.P, p_begin + p.p_per_split);
  const int affine = p.affine;
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, (short)0, (int)p.dybytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.xbytes, 0x00020000);
  constexpr unsigned OOB = 0xFFFFFFF0u;
  // every step is full when P is a multiple of BP (p_per_split always is): no row masks at all
  const bool exact = (p.P % BP) == 0;

  // ---- A (dY) slots: fixed column; element offsets advance by BP rows per step ----
  const int a_col = tid % A_CPR;
  const int a_n = n0 + a_col * 8;
  const bool a_col_ok = a_n < p.Cout;
  // Gram mode: dY is the same BN-ReLU input as x (affine on both operands) + column sums
  const bool dy_aff = p.dy_affine != 0;
  const uint32_t rfloor = affine == 2 ? 0u : 0x80008000u;   // packed ReLU floor (int16 min = no ReLU)
  float dsc[8], dsh[8], csum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    dsc[e] = (dy_aff && a_col_ok) ? p.in_scale[a_n + e] : 0.f;
    dsh[e] = (dy_aff && a_col_ok) ? p.in_shift[a_n + e] : 0.f;
    csum[e] = 0.f;
  }
  const bool do_csum = dy_aff && p.colsum != nullptr && kt_idx == 0;
  unsigned ra_valid = ~0u;
  int a_vo[A_SLOTS], a_row[A_SLOTS], sa[A_SLOTS];
#pragma unroll
  for (int s = 0; s < A_SLOTS; ++s) {
    const int idx = tid + s * NT;
    a_row[s] = idx / A_CPR;
    // element offset of the slot's dY row (DENSE: byte offset for the buffer loads; columns past Cout
    // read a real, ignored address — those dW rows are never stored)
    a_vo[s] = (p_begin + a_row[s]) * p.ldd + a_n;
    if constexpr (DENSE) a_vo[s] = (idx < A_CHUNKS && a_col_ok) ? a_vo[s] * 2 : 0;
    sa[s] = img_off<BMW>(a_row[s], a_col * 16);
  }

  // ---- B (im2col) slots: fixed (tap, cin) column per block; positions advance by BP ----
  const int b_col = tid % B_CPR;
  const int kb = k0 + b_col * CH;
  const bool b_col_ok = kb < p.K;
  int b_dt = 0, b_dh = 0, b_dw = 0, b_c = 0;
  if (b_col_ok) {
    const int tap = kb / p.Cin;
    b_c = kb - tap * p.Cin;
    b_dt = tap / (p.kh * p.kw);
    const int r = tap - b_dt * p.kh * p.kw;
    b_dh = r / p.kw;
    b_dw = r - b_dh * p.kw;
  }
  const int tapoff = ((b_dt * p.Hi + b_dh) * p.Wi + b_dw) * p.ldx + b_c;
  // the block's im2col column is fixed, so this thread's 8 BN scale/shift values are too: registers
  float asc[CH], ash[CH];
#pragma unroll
  for (int e = 0; e < CH; ++e) {
    asc[e] = (affine && b_col_ok) ? p.in_scale[b_c + e] : 0.f;
    ash[e] = (affine && b_col_ok) ? p.in_shift[b_c + e] : 0.f;
  }
  const bool check = p.pt | p.ph | p.pw;   // taps can only leave the tensor through padding
  // per-slot output position (pb, pt, ph, pw) and its input origin (bt, bh, bw) / linear offset bio
  const int OHW = p.Ho * p.Wo, OTHW = p.To * OHW;
  int pt_[B_SLOTS], ph_[B_SLOTS], pw_[B_SLOTS], bt[B_SLOTS], bh[B_SLOTS], bw[B_SLOTS], bio[B_SLOTS],
      b_row[B_SLOTS], sb[B_SLOTS];
  // offset deltas of the incremental walk
  const int dW1 = BP * p.sw * p.ldx;
  const int dWrap = (p.sh * p.Wi - p.Wo * p.sw) * p.ldx;
  const int dHrap = (p.st * p.Hi * p.Wi - p.Ho * p.sh * p.Wi) * p.ldx;
  const int dTrap = (p.Ti * p.Hi * p.Wi - p.To * p.st * p.Hi * p.Wi) * p.ldx;
#pragma unroll
  for (int s = 0; s < B_SLOTS; ++s) {
    b_row[s] = (tid + s * NT) / B_CPR;
    int q = p_begin + b_row[s];
    const int b = q / OTHW; q -= b * OTHW;
    const int t = q / OHW; q -= t * OHW;
    const int h = q / p.Wo;
    pt_[s] = t; ph_[s] = h; pw_[s] = q - h * p.Wo;
    bt[s] = t * p.st - p.pt; bh[s] = h * p.sh - p.ph; bw[s] = pw_[s] * p.sw - p.pw;
    bio[s] = ((b * p.Ti + bt[s]) * p.Hi + bh[s]) * p.Wi * p.ldx + bw[s] * p.ldx;
    sb[s] = img_off<BNW>(b_row[s], b_col * CH * 2);
  }
  auto advance_pos = [&](int s) {
    pw_[s] += BP; bw[s] += BP * p.sw; bio[s] += dW1;
    while (pw_[s] >= p.Wo) {
      pw_[s] -= p.Wo; bw[s] -= p.Wo * p.sw; bh[s] += p.sh; bio[s] += dWrap;
      if (++ph_[s] == p.Ho) {
        ph_[s] = 0; bh[s] -= p.Ho * p.sh; bt[s] += p.st; bio[s] += dHrap;
        if (++pt_[s] == p.To) { pt_[s] = 0; bt[s] -= p.To * p.st; bio[s] += dTrap; }
      }
    }
  };

  uint4 ra[A_SLOTS];
  VT rb[B_SLOTS];
  unsigned rb_valid = 0;
  int pcur = p_begin;

  int b_vo[B_SLOTS];
#pragma unroll
  for (int s = 0; s < B_SLOTS; ++s)
    b_vo[s] = (DENSE && tid + s * NT < B_CHUNKS && b_col_ok) ? ((p_begin + b_row[s]) * p.ldx + b_c) * 2 : 0;

  auto load = [&]() {
    const int pd = pcur - p_begin;  // uniform step offset (positions)
    rb_valid = 0;
    if (dy_aff) {   // rows past this split (or P): act(0) != 0, so both Gram operands are zeroed there
      ra_valid = 0;
#pragma unroll
      for (int s = 0; s < A_SLOTS; ++s) ra_valid |= (pcur + a_row[s] < p_end ? 1u : 0u) << s;
    }
    if constexpr (DENSE && CH == 8) {
#pragma unroll
      for (int s = 0; s < A_SLOTS; ++s) {
        if (exact) {
          ra[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(dyr, a_vo[s], pd * p.ldd * 2, 0));
        } else {
          const bool v = pcur + a_row[s] < p_end;
          ra[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
              dyr, v ? a_vo[s] + pd * p.ldd * 2 : (int)OOB, 0, 0));
        }
      }
#pragma unroll
      for (int s = 0; s < B_SLOTS; ++s) {
        if (exact) {
          rb[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, b_vo[s], pd * p.ldx * 2, 0));
        } else {
          const bool v = pcur + b_row[s] < p_end;
          rb[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
              xr, v ? b_vo[s] + pd * p.ldx * 2 : (int)OOB, 0, 0));
        }
      }
      rb_valid = dy_aff ? 0u : ~0u;
      if (dy_aff) {
#pragma unroll
        for (int s = 0; s < B_SLOTS; ++s) rb_valid |= (pcur + b_row[s] < p_end ? 1u : 0u) << s;
      }
      pcur += BP;
      return;
    }
#pragma unroll
    for (int s = 0; s < A_SLOTS; ++s) {
      if (tid + s * NT < A_CHUNKS && a_col_ok && pcur + a_row[s] < p_end)
        ra[s] = *reinterpret_cast<const uint4*>(p.dy + a_vo[s]);
      else
        ra[s] = uint4{0, 0, 0, 0};
      a_vo[s] += BP * p.ldd;
    }
#pragma unroll
    for (int s = 0; s < B_SLOTS; ++s) {
      bool v = (tid + s * NT < B_CHUNKS) & b_col_ok & (pcur + b_row[s] < p_end);   // '&': no branch per term
      if (check)
        v = v & ((unsigned)(bt[s] + b_dt) < (unsigned)p.Ti) & ((unsigned)(bh[s] + b_dh) < (unsigned)p.Hi) &
            ((unsigned)(bw[s] + b_dw) < (unsigned)p.Wi);
      if (v) {
        rb[s] = *reinterpret_cast<const VT*>(p.x + (bio[s] + tapoff));
        rb_valid |= 1u << s;
      } else {
        rb[s] = VT{};
      }
      advance_pos(s);
    }
    pcur += BP;
  };

  auto store_lds = [&](int buf) {
    char* A = smem + buf * TILE;
    char* B = A + A_BYTES;
#pragma unroll
    for (int s = 0; s < A_SLOTS; ++s) {
      if constexpr (A_CHUNKS % NT != 0) if (tid + s * NT >= A_CHUNKS) break;
      uint4 v = ra[s];
      if (dy_aff) {   // packed: FMAs, cvt_pk, v_pk_max_i16 against the uniform floor, row mask
        float f[8];
        unpack8(v, f);
        const uint32_t keep = 0u - ((ra_valid >> s) & 1u);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = __builtin_fmaf(f[e], dsc[e], dsh[e]);
        v = pack8_fast(f);
        v = make_uint4(max_e16x2(v.x, rfloor) & keep, max_e16x2(v.y, rfloor) & keep,
                       max_e16x2(v.z, rfloor) & keep, max_e16x2(v.w, rfloor) & keep);
        if (do_csum) {   // sum of the bf16 operand values actually multiplied
          float q[8];
          unpack8(v, q);
#pragma unroll
          for (int e = 0; e < 8; ++e) csum[e] += q[e];
        }
      }
      *reinterpret_cast<uint4*>(A + sa[s]) = v;
    }
#pragma unroll
    for (int s = 0; s < B_SLOTS; ++s) {
      if constexpr (B_CHUNKS % NT != 0) if (tid + s * NT >= B_CHUNKS) break;
      VT v = rb[s];
      const uint32_t keep = 0u - ((rb_valid >> s) & 1u);   // padding stays zero (all ones on the dense path)
      if (affine) {
        // recompute the producer's BN(+ReLU) on the fly: packed cvt + v_pk_max_i16 against the uniform floor
        float f[CH];
        if constexpr (CH == 8) unpack8(v, f); else unpack4(v, f);
#pragma unroll
        for (int e = 0; e < CH; ++e) f[e] = __builtin_fmaf(f[e], asc[e], ash[e]);
        if constexpr (CH == 8) {
          v = pack8_fast(f);
          v = make_uint4(max_e16x2(v.x, rfloor) & keep, max_e16x2(v.y, rfloor) & keep,
                         max_e16x2(v.z, rfloor) & keep, max_e16x2(v.w, rfloor) & keep);
        } else {
          v = make_uint2(max_e16x2(cvt_pk_e16(f[0], f[1]), rfloor) & keep,
                         max_e16x2(cvt_pk_e16(f[2], f[3]), rfloor) & keep);
        }
      }
      *reinterpret_cast<VT*>(B + sb[s]) = v;
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nsteps = (p_end - p_begin + BP - 1) / BP;
  // one-stage-ahead register ring (as conv_igemm.hip): stage s+1 is written right after the barrier of
  // step s and stage s+2 issued at once, so each load has a whole step of MFMA work to land
  if (nsteps > 0) {
    load();
    store_lds(0);
  }
  if (nsteps > 1) load();

  // tr-read addressing: group g = lane>>4 covers p rows 8g..8g+7; lane i = lane&15 supplies row
  // (i>>2) of a 4-row block and columns 4*(i&3)..+3 of the 16-column block.  Offsets precomputed.
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
  auto frags = [&](const char* A, int kk, ev8_t (&af)[TM], ev8_t (&bfr)[TN]) {   // rows 32*kk.. of the stage
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
  };
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    __syncthreads();
    const char* A = smem + cur * TILE;
    // the stage's first fragments are read BEFORE the next stage is staged: their LDS latency overlaps the
    // staging work (the recomputed BN-ReLU of the im2col operand, ds_write), which the MFMAs otherwise waited out
    // (not for the largest tiles, whose registers are already spoken for: there it spills)
    constexpr bool HOIST = BMW * BNW <= 256 * 128 && !(CH == 4 && BNW == 256);
    ev8_t af[TM], bfr[TN];
    if constexpr (HOIST) frags(A, 0, af, bfr);
    if (step + 1 < nsteps) {
      store_lds(cur ^ 1);
      if (step + 2 < nsteps) load();
    }
#pragma unroll
    for (int kk = 0; kk < BP / 32; ++kk) {
      if (kk > 0 || !HOIST) frags(A, kk, af, bfr);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = PVA_MFMA16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  if (do_csum) {
    // threads with the same A column (tid % A_CPR) hold partial sums of the same 8 channels: reduce within
    // the wave, then across waves through the (now idle) LDS in a fixed order -> colsum[split][n]
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    constexpr int NWAVE = NT / 64;
    static_assert(A_CPR <= 64, "column groups per wave");
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = wave_sum_stride(csum[e], A_CPR);
    if (lane < A_CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wid * BMW + a_col * 8 + e] = csum[e];
    }
    __syncthreads();
    for (int c = tid; c < BMW; c += NT) {
      float t = 0.f;
      for (int w = 0; w < NWAVE; ++w) t += red[w * BMW + c];
      if (n0 + c < p.Cout) p.colsum[(int64_t)split * p.Cout + n0 + c] = t;
    }
  }

  // D[n][k]: lane holds k = col (lane&15), n = 4*(lane>>4) + r.  With one slab the tile is stored;
  // with several, slabs accumulate into one zero-initialised fp32 buffer with no-return
  // global_atomic_add_f32 (each wave-instruction = 4 rows x 64 contiguous bytes).
  // deterministic (slab) mode: every split stores its own slab; the convert kernel sums them in order
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

// ------------------------------------------------------------------------------------------------
// Narrow weight gradient (Cout <= 16 * MT, K = taps x Cin <= 16 * NTN, Cin % 8 == 0): the fast-pathway
// convs, whose block tiles above spend their time in per-stage barriers.  Every WAVE is an independent
// worker over its own contiguous position range with a private LDS slice, so there is no workgroup barrier
// at all: lane l stages row l of a 64-position chunk — its dY row (A image) and its im2col row, one 16-B
// chunk per (tap, 8 channels) (B image) — and the wave reads the two 32-row halves back with
// ds_read_b64_tr_b16 for 2 x MT x NTN MFMAs.  LDS ops of one wave execute in order, so the reads see the
// writes and the next chunk's writes never overtake them.  The next chunk's global loads are issued before
// the current chunk's MFMAs.  Tiles are added into the zeroed fp32 accumulator with no-return atomics.
// Gram mode (dy_affine) applies the x affine to dY too and writes per-wave column sums (slab row = wave).
template <int MT, int NTN>
__global__ __launch_bounds__(256) void wgrad_narrow_kernel(const WgradParams p) {
  constexpr int KP = 16 * NTN, MP = 16 * MT;
  constexpr int KC = KP / 8, MC = MP / 8;          // 16-B chunks per im2col / dY row (upper bounds)
  constexpr int A_IMG = 64 * MP * 2, B_IMG = 64 * KP * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + wave;
  if (gw >= p.splits) return;   // grid rounded up to whole workgroups; no workgroup barriers follow
  char* A = smem + wave * (A_IMG + B_IMG);
  char* B = A + A_IMG;
  const int p_begin = gw * p.p_per_split;
  const int p_end = min(p.P, p_begin + p.p_per_split);
  const int kchunks = p.K / 8, mchunks = (p.Cout + 7) / 8;
  const int affine = p.affine;
  const bool dy_aff = p.dy_affine != 0;
  f32x4_t acc[MT][NTN];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float csum[MP];
#pragma unroll
  for (int e = 0; e < MP; ++e) csum[e] = 0.f;
  const int OHW = p.Ho * p.Wo, OTHW = p.To * OHW;
  const bool check = p.pt | p.ph | p.pw;
  // transposed-read addressing (as conv_wgrad_kernel): group g = lane>>4 covers rows 8g..8g+7 of a
  // 32-row half; lane i = lane&15 supplies row (i>>2) of a 4-row block, columns 4*(i&3)..+3
  const int g = lane >> 4, li = lane & 15;
  const int tr_row = 8 * g + (li >> 2);
  const int tr_colb = (li & 3) * 8;
  uint4 ra[MC], rb[KC];
  // the im2col chunk kc = (tap, 8 channels) is the same for every position: decode it once (dt | dh << 4 | dw << 8 |
  // c0 << 12, and its element offset from the position's base) instead of three divisions per chunk and position
  int kcode[KC], ktoff[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    const int k = kc * 8;
    const int tap = k / p.Cin, c0 = k - tap * p.Cin;
    const int dt = tap / (p.kh * p.kw), r = tap - dt * p.kh * p.kw;
    const int dh = r / p.kw, dw = r - dh * p.kw;
    kcode[kc] = dt | (dh << 4) | (dw << 8) | (c0 << 12);
    ktoff[kc] = ((dt * p.Hi + dh) * p.Wi + dw) * p.ldx + c0;
  }
  auto act8 = [&](uint4 v, const float* sc, const float* sh) {
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float z = __builtin_fmaf(f[e], sc[e], sh[e]);
      f[e] = affine == 2 ? fmaxf(z, 0.f) : z;
    }
    return pack8_fast(f);
  };
  auto load = [&](int pbase) {
    const int pp = pbase + lane;
#pragma unroll
    for (int mc = 0; mc < MC; ++mc) ra[mc] = uint4{0, 0, 0, 0};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) rb[kc] = uint4{0, 0, 0, 0};
    if (pp >= p_end) return;   // rows past the range stay zero in both images (also in Gram mode)
    const uint16_t* dyr = p.dy + (int64_t)pp * p.ldd;
#pragma unroll
    for (int mc = 0; mc < MC; ++mc)
      if (mc < mchunks) ra[mc] = *reinterpret_cast<const uint4*>(dyr + mc * 8);
    int q = pp;
    const int b = pva_fdiv(q, p.mg_othw, p.sh_othw); q -= b * OTHW;
    const int t = pva_fdiv(q, p.mg_ohw, p.sh_ohw); q -= t * OHW;
    const int h = pva_fdiv(q, p.mg_wo, p.sh_wo), w = q - h * p.Wo;
    const int bt = t * p.st - p.pt, bh = h * p.sh - p.ph, bw = w * p.sw - p.pw;
    const uint16_t* xb = p.x + ((((int64_t)b * p.Ti + bt) * p.Hi + bh) * p.Wi + bw) * p.ldx;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      if (kc < kchunks) {
        const int dt = kcode[kc] & 15, dh = (kcode[kc] >> 4) & 15, dw = (kcode[kc] >> 8) & 15;
        bool v = true;
        if (check)
          v = (unsigned)(bt + dt) < (unsigned)p.Ti && (unsigned)(bh + dh) < (unsigned)p.Hi &&
              (unsigned)(bw + dw) < (unsigned)p.Wi;
        if (v) {
          rb[kc] = *reinterpret_cast<const uint4*>(xb + ktoff[kc]);
          if (affine) {   // padding stays zero
            const int c0 = kcode[kc] >> 12;
            rb[kc] = act8(rb[kc], p.in_scale + c0, p.in_shift + c0);
          }
        }
      }
    }
    if (dy_aff) {   // Gram mode: dY is the same activation (Cout = Cin channels)
#pragma unroll
      for (int mc = 0; mc < MC; ++mc)
        if (mc < mchunks) ra[mc] = act8(ra[mc], p.in_scale + mc * 8, p.in_shift + mc * 8);
    }
  };
  const int niter = (p_end - p_begin + 63) / 64;
  if (niter > 0) load(p_begin);
  for (int it = 0; it < niter; ++it) {
    // stage this chunk (row = lane) into the wave's private images
#pragma unroll
    for (int mc = 0; mc < MC; ++mc) *reinterpret_cast<uint4*>(A + img_off<MP>(lane, mc * 16)) = ra[mc];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) *reinterpret_cast<uint4*>(B + img_off<KP>(lane, kc * 16)) = rb[kc];
    if (dy_aff && p.colsum) {
#pragma unroll
      for (int mc = 0; mc < MC; ++mc) {
        float f[8];
        unpack8(ra[mc], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[mc * 8 + e] += f[e];
      }
    }
    if (it + 1 < niter) load(p_begin + (it + 1) * 64);   // next chunk's loads fly under the MFMAs
#pragma unroll
    for (int hlf = 0; hlf < 2; ++hlf) {
      const int rb0 = hlf * 32;
      ev8_t af[MT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const s16x4_t lo = tr_read(A + img_off<MP>(rb0 + tr_row, i * 32 + tr_colb));
        const s16x4_t hi = tr_read(A + img_off<MP>(rb0 + tr_row + 4, i * 32 + tr_colb));
        af[i] = __builtin_bit_cast(ev8_t, (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
      }
#pragma unroll
      for (int j = 0; j < NTN; ++j) {
        const s16x4_t blo = tr_read(B + img_off<KP>(rb0 + tr_row, j * 32 + tr_colb));
        const s16x4_t bhi = tr_read(B + img_off<KP>(rb0 + tr_row + 4, j * 32 + tr_colb));
        const ev8_t bf = __builtin_bit_cast(ev8_t,
                                               (s16x8_t){blo[0], blo[1], blo[2], blo[3], bhi[0], bhi[1], bhi[2], bhi[3]});
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i][j] = PVA_MFMA16(af[i], bf, acc[i][j], 0, 0, 0);
      }
    }
  }
  // D[n][k]: lane holds k = j*16 + (lane&15), n = i*16 + 4*(lane>>4) + r
  if (niter > 0) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NTN; ++j) {
        const int k = j * 16 + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = i * 16 + 4 * g + r;
          if (n < p.Cout && k < p.K) atomicAdd(p.partial + (int64_t)n * p.K + k, acc[i][j][r]);
        }
      }
  }
  if (dy_aff && p.colsum) {
#pragma unroll
    for (int e = 0; e < MP; ++e) csum[e] = wave_sum(csum[e]);
    if (lane < p.Cout) {
      float v = 0.f;
#pragma unroll
      for (int e = 0; e < MP; ++e) v = lane == e ? csum[e] : v;
      p.colsum[(int64_t)gw * p.Cout + lane] = v;
    }
  }
}

template <int MT, int NTN>
void launch_narrow(const WgradParams& p0, hipStream_t stream) {
  WgradParams p = p0;
  pva_magic_div(p.To * p.Ho * p.Wo, &p.mg_othw, &p.sh_othw);
  pva_magic_div(p.Ho * p.Wo, &p.mg_ohw, &p.sh_ohw);
  pva_magic_div(p.Wo, &p.mg_wo, &p.sh_wo);
  const int blocks = (p.splits + 3) / 4;
  const size_t lds = 4 * (64 * 16 * MT * 2 + 64 * 16 * NTN * 2);
  hipLaunchKernelGGL((wgrad_narrow_kernel<MT, NTN>), dim3(blocks), dim3(256), lds, stream, p);
}

template <int MT>
void launch_narrow_k(const WgradParams& p, hipStream_t stream) {
  switch ((p.K + 15) / 16) {
    case 1: launch_narrow<MT, 1>(p, stream); break;
    case 2: launch_narrow<MT, 2>(p, stream); break;
    case 3: launch_narrow<MT, 3>(p, stream); break;
    case 4: launch_narrow<MT, 4>(p, stream); break;
    case 5: launch_narrow<MT, 5>(p, stream); break;
    case 6: launch_narrow<MT, 6>(p, stream); break;
    case 7: launch_narrow<MT, 7>(p, stream); break;
    default: launch_narrow<MT, 8>(p, stream); break;
  }
}

template <int BMW, int BNW, int WMW, int WNW, int CH, int BP>
void launch_w(const WgradParams& p, hipStream_t stream) {
  constexpr int NT = (BMW / WMW) * (BNW / WNW) * 64;
  const dim3 grid(((p.Cout + BMW - 1) / BMW) * ((p.K + BNW - 1) / BNW) * p.splits);
  const size_t lds = 2 * BP * (BMW + BNW) * 2;
  const bool dense = p.kt == 1 && p.kh == 1 && p.kw == 1 && p.st == 1 && p.sh == 1 && p.sw == 1 &&
                     p.pt == 0 && p.ph == 0 && p.pw == 0;
  if constexpr (CH == 8) {
    if (dense) {
      hipLaunchKernelGGL((conv_wgrad_kernel<BMW, BNW, WMW, WNW, CH, 1, BP>), grid, dim3(NT), lds, stream, p);
      return;
    }
  }
  hipLaunchKernelGGL((conv_wgrad_kernel<BMW, BNW, WMW, WNW, CH, 0, BP>), grid, dim3(NT), lds, stream, p);
}

// tiles 0-3: narrow outputs (fast pathway, small Cout); 4-7: 64x64 / 128x64 per wave (TM x TN = 16 or 32
// MFMAs per 32-position k-step against 16 / 24 transposed LDS reads) for the compute-bound slow-pathway
// weight gradients (Cout >= 128, K = taps x Cin >= 576)
template <int CH, int BP>
void launch_w_variant(int v, const WgradParams& p, hipStream_t stream) {
  switch (v) {
    case 0: launch_w<16, 128, 16, 32, CH, BP>(p, stream); break;
    case 1: launch_w<32, 128, 32, 32, CH, BP>(p, stream); break;
    case 2: launch_w<64, 64, 32, 32, CH, BP>(p, stream); break;
    case 3: launch_w<128, 64, 64, 32, CH, BP>(p, stream); break;
    case 4: launch_w<128, 128, 64, 64, CH, BP>(p, stream); break;
    case 5: launch_w<256, 128, 64, 64, CH, BP>(p, stream); break;
    case 6: launch_w<128, 256, 64, 64, CH, BP>(p, stream); break;
    default: launch_w<256, 256, 128, 64, CH, BP>(p, stream); break;
  }
}

// dW accumulator [Cout][taps][Cin_pad] -> grad[Cout][Cin][taps] (PyTorch layout),
// grad = beta * grad + scale * acc ; the accumulator is re-zeroed for the next layer (atomic mode).
__global__ void wgrad_convert_kernel(float* __restrict__ accbuf, float* __restrict__ grad, int total,
                                     int taps, int Cin, int Cin_real, float scale, float beta, int rezero,
                                     int slabs, int64_t slab_stride) {
  const int per_n = Cin_real * taps;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
    const int n = o / per_n;
    const int rem = o - n * per_n;
    const int c = rem / taps;
    const int tap = rem - c * taps;
    const int a = (n * taps + tap) * Cin + c;
    float v = accbuf[a];
    for (int s = 1; s < slabs; ++s) v += accbuf[s * slab_stride + a];  // fixed order
    if (rezero) accbuf[a] = 0.f;
    grad[o] = (beta == 0.f ? 0.f : beta * grad[o]) + scale * v;
  }
}

// slab mode: 256 consecutive accumulator entries per block (4 per lane, 16-B loads); wave w sums the slabs
// s = w, w + NW, ... (four running partials, fixed order), the NW wave partials are combined in wave order through
// LDS.  Fixed order for a given slab count, 4*NW 16-B loads in flight per lane (one float per lane per load ran
// these at ~0.5 TB/s: the BN-fold G products reduce up to 4096 slabs).
template <int NW>
__global__ __launch_bounds__(NW * 64) void wgrad_slab_reduce_kernel(const float* __restrict__ acc,
                                                                    float* __restrict__ grad, int total_a, int taps,
                                                                    int Cin, int Cin_real, float scale, float beta,
                                                                    int slabs, int64_t ss) {
  __shared__ f32x4_t red[NW][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int a = (blockIdx.x * 64 + lane) * 4;   // total_a and ss are multiples of 4 (Cin % 8 == 0)
  f32x4_t v = {0.f, 0.f, 0.f, 0.f};
  if (a < total_a) {
    const f32x4_t* base = reinterpret_cast<const f32x4_t*>(acc + a);
    const int64_t s4 = ss >> 2;
    f32x4_t t0 = v, t1 = v, t2 = v, t3 = v;
    int s = w;
    for (; s + 3 * NW < slabs; s += 4 * NW) {
      t0 += base[(int64_t)s * s4];
      t1 += base[(int64_t)(s + NW) * s4];
      t2 += base[(int64_t)(s + 2 * NW) * s4];
      t3 += base[(int64_t)(s + 3 * NW) * s4];
    }
    for (; s < slabs; s += NW) t0 += base[(int64_t)s * s4];
    v = (t0 + t1) + (t2 + t3);
  }
  if constexpr (NW > 1) {
    red[w][lane] = v;
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int i = 1; i < NW; ++i) v += red[i][lane];
  }
  if (a >= total_a) return;
  const int per_n = taps * Cin;
  const int n = a / per_n;
  const int rem = a - n * per_n;
  const int tap = rem / Cin;
  const int c = rem - tap * Cin;   // 4 consecutive channels of one (n, tap)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (c + e >= Cin_real) break;
    const int o = (n * Cin_real + c + e) * taps + tap;
    grad[o] = (beta == 0.f ? 0.f : beta * grad[o]) + scale * v[e];
  }
}

}  // namespace

// Shape-based tile choice: (BMW over cout, BNW over k).
static int wgrad_variant(int Cout, int K) {
  if (Cout <= 16) return 0;   // 16 x 128
  if (Cout <= 32) return 1;   // 32 x 128
  if (Cout <= 64) return 2;   // 64 x 64
  return 3;                   // 128 x 64
}

static int wgrad_tile_index(int variant) { return (variant & 3) | ((variant >> 3) & 1) << 2; }

void conv_wgrad_tile(int Cout, int K, int variant, int* bmw, int* bnw) {
  switch (variant >= 0 ? wgrad_tile_index(variant) : wgrad_variant(Cout, K)) {
    case 0: *bmw = 16; *bnw = 128; break;
    case 1: *bmw = 32; *bnw = 128; break;
    case 2: *bmw = 64; *bnw = 64; break;
    case 3: *bmw = 128; *bnw = 64; break;
    case 4: *bmw = 128; *bnw = 128; break;
    case 5: *bmw = 256; *bnw = 128; break;
    case 6: *bmw = 128; *bnw = 256; break;
    default: *bmw = 256; *bnw = 256; break;
  }
}

// p.variant: -1 = heuristic tile, 32-position stages; else bits 0-1 (+ bit 3 for tiles 4-7) = tile variant,
// bit 2 = 64-position stages (p_per_split must then be a multiple of 64)
// narrow kernel legality: Cout <= 32, Cin % 8 == 0, K <= 128
int wgrad_narrow_legal(int Cout, int Cin, int K) { return (Cout <= 32 && Cin % 8 == 0 && K <= 128) ? 1 : 0; }

int wgrad_halo_legal(const WgradParams& p);
void wgrad_halo_launch(const WgradParams& p, hipStream_t s);

void wgrad_box_launch(const WgradParams& p, hipStream_t st);

// row-table kernel (wgrad_rt_impl.h): 16-B chunks on both operands, tiles 2-7, no Gram mode
int wgrad_rt_legal(int Cout, int Cin, int ldd, int ldx, int chunk, int dy_affine) {
  return (chunk == 8 && Cin % 8 == 0 && Cout % 8 == 0 && ldd % 8 == 0 && ldx % 8 == 0 && !dy_affine) ? 1 : 0;
}

void wgrad_rt_run_a0(int v, bool bp64, bool check, const wgrad_rt::RtParams& rp, hipStream_t st);
void wgrad_rt_run_a1(int v, bool bp64, bool check, const wgrad_rt::RtParams& rp, hipStream_t st);

void conv_wgrad_launch(const WgradParams& p, int chunk, hipStream_t stream) {
  if (p.variant >= 0 && (p.variant & (1 << 25))) {   // row-table kernel; legality checked by the binding
    wgrad_rt::RtParams rp;
    rp.p = p;
    wgrad_rt::magic_div(p.Wo, &rp.mWo, &rp.sWo1, &rp.sWo2);
    wgrad_rt::magic_div(p.Ho, &rp.mHo, &rp.sHo1, &rp.sHo2);
    wgrad_rt::magic_div(p.To, &rp.mTo, &rp.sTo1, &rp.sTo2);
    const int v = wgrad_tile_index(p.variant);
    const bool bp64 = p.variant & 4;
    const bool check = p.pt | p.ph | p.pw;
    if (p.affine) wgrad_rt_run_a1(v < 2 ? 2 : v, bp64, check, rp, stream);
    else wgrad_rt_run_a0(v < 2 ? 2 : v, bp64, check, rp, stream);
    return;
  }
  if (p.variant >= 0 && (p.variant & (1 << 26))) {   // box-staged (1,3,3) kernel (wgrad_box.hip): per-split slabs
    wgrad_box_launch(p, stream);
    return;
  }
  if (p.variant >= 0 && (p.variant & 32)) {   // halo-staged kernel (wgrad_halo.hip); legality checked by the binding
    wgrad_halo_launch(p, stream);
    return;
  }
  if (p.variant >= 0 && (p.variant & 16)) {   // narrow per-wave kernel: p.splits = waves, p_per_split = rows/wave
    if (p.Cout <= 16) launch_narrow_k<1>(p, stream); else launch_narrow_k<2>(p, stream);
    return;
  }
  const int v = p.variant >= 0 ? wgrad_tile_index(p.variant) : wgrad_variant(p.Cout, p.K);
  const bool bp64 = p.variant >= 0 && (p.variant & 4);
  if (chunk == 8) {
    if (bp64) launch_w_variant<8, 64>(v, p, stream); else launch_w_variant<8, 32>(v, p, stream);
  } else {
    if (bp64) launch_w_variant<4, 64>(v, p, stream); else launch_w_variant<4, 32>(v, p, stream);
  }
}

void wgrad_reduce_launch(float* accbuf, float* grad, int splits, int Cout, int taps, int Cin, int Cin_real,
                         float scale, float beta, int slab, hipStream_t stream) {
  // atomic mode: one accumulator, re-zeroed here; slab mode: `splits` slabs fully overwritten by the kernel
  if (slab && splits > 1 && Cin % 4 == 0) {   // (Cin % 4 != 0: the per-element pass below sums the slabs)
    const int total_a = Cout * taps * Cin;
    const dim3 grid((total_a / 4 + 63) / 64);
    const int64_t ss = (int64_t)Cout * taps * Cin;
#define PVA_SLAB_RED(NW) \
    hipLaunchKernelGGL(wgrad_slab_reduce_kernel<NW>, grid, dim3(NW * 64), 0, stream, accbuf, grad, total_a, taps, Cin, \
                       Cin_real, scale, beta, splits, ss)
    if (splits >= 128) PVA_SLAB_RED(16);
    else if (splits >= 32) PVA_SLAB_RED(8);
    else if (splits >= 8) PVA_SLAB_RED(4);
    else PVA_SLAB_RED(1);
#undef PVA_SLAB_RED
    return;
  }
  const int total = Cout * taps * Cin_real;
  int blocks = std::min((total + 255) / 256, 4096);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(wgrad_convert_kernel, dim3(blocks), dim3(256), 0, stream, accbuf, grad, total, taps, Cin,
                     Cin_real, scale, beta, slab ? 0 : 1, slab ? splits : 1, (int64_t)Cout * taps * Cin);
}

PVA_NS_END  // namespace PVA_NS
