// Shared device helpers for the gfx950 (CDNA4) kernels of pytorchvideo_accelerate_amd.
// Everything here is written for 64-lane wavefronts and the MFMA 16x16x32 bf16/f16 operand maps
// (cdna_hip_programming.md §3: lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15];
//  D: col = l&15, row = 4(l>>4)+r).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Compute element type of the translation unit.  Every kernel source is compiled twice (pytorchvideo_accelerate_amd/
// _build.py): PVA_F16=0 -> bf16 operands in namespace pva_bf16, PVA_F16=1 -> fp16 operands in namespace pva_f16
// (same kernels, same fp32 accumulation; v_mfma_f32_16x16x32_f16 runs at the bf16 instruction's rate).  The
// bindings pick the namespace by the dtype of the 16-bit tensors (csrc/kernels/launchers.h).
#ifndef PVA_F16
#define PVA_F16 0
#endif
#if PVA_F16
#define PVA_NS pva_f16
typedef _Float16 e16s_t;                                   // arithmetic type of one element
#define PVA_MFMA16 __builtin_amdgcn_mfma_f32_16x16x32_f16
#else
#define PVA_NS pva_bf16
typedef __bf16 e16s_t;
#define PVA_MFMA16 __builtin_amdgcn_mfma_f32_16x16x32_bf16
#endif
#define PVA_NS_BEGIN namespace PVA_NS {
#define PVA_NS_END }

typedef uint16_t e16_t;  // storage type of a 16-bit element (bf16 or fp16 per build)
typedef __attribute__((ext_vector_type(8))) e16s_t ev8_t;  // MFMA 16x16x32 A/B operand
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) e16s_t ev2_t;
typedef __attribute__((ext_vector_type(2))) short s16x2_t;

#define PVA_WAVE 64
#define PVA_NXCD 8

// element -> f32 (exact) for a lone element and for the low / high element of a packed pair
#if PVA_F16
__device__ __forceinline__ float e2f(e16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
__device__ __forceinline__ float lo2f(uint32_t w) { return e2f((e16_t)(w & 0xffffu)); }
__device__ __forceinline__ float hi2f(uint32_t w) { return e2f((e16_t)(w >> 16)); }
#else
__device__ __forceinline__ float e2f(e16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ float lo2f(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi2f(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
#endif

// Round-to-nearest-even with NaN preserved (hipcc lowers the bf16 cast to v_cvt_pk_bf16_f32; fp16 overflows to inf,
// which the fp16 loss scaler detects in the weight gradients).
__device__ __forceinline__ e16_t f2e(float f) {
  e16s_t b = (e16s_t)f;
  return __builtin_bit_cast(e16_t, b);
}

// 2 x f32 -> packed pair in ONE conversion instruction (v_cvt_pk_bf16_f32; RNE, NaN-preserving).  Two scalar
// casts OR-ed together cost 2 cvt + 4 mask/shift/or VALU ops per pair (measured in the ISA): the packing sits in
// every epilogue and elementwise kernel, so it matters.
__device__ __forceinline__ uint32_t cvt_pk_e16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, ev2_t));
}

__device__ __forceinline__ uint32_t pack2(float a, float b) { return cvt_pk_e16(a, b); }

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = lo2f(v.x); f[1] = hi2f(v.x);
  f[2] = lo2f(v.y); f[3] = hi2f(v.y);
  f[4] = lo2f(v.z); f[5] = hi2f(v.z);
  f[6] = lo2f(v.w); f[7] = hi2f(v.w);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}


__device__ __forceinline__ uint4 pack8_fast(const float* f) {
  return make_uint4(cvt_pk_e16(f[0], f[1]), cvt_pk_e16(f[2], f[3]), cvt_pk_e16(f[4], f[5]), cvt_pk_e16(f[6], f[7]));
}

// ReLU on packed 16-bit floats: bf16 and fp16 are sign-magnitude, so max as signed int16 against 0 zeroes every
// negative (and -0) lane and keeps positives: one v_pk_max_i16 per pair.
__device__ __forceinline__ uint32_t relu_e16x2(uint32_t w) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2_t, w), (s16x2_t){0, 0}));
}

__device__ __forceinline__ uint4 relu_e16x8(const uint4& v) {
  return make_uint4(relu_e16x2(v.x), relu_e16x2(v.y), relu_e16x2(v.z), relu_e16x2(v.w));
}

// The same max against a run-time floor pair: floor 0 is the ReLU, floor 0x80008000 (int16 minimum in both lanes)
// keeps every value — a wave-uniform switch between BN and BN+ReLU without a select per element.
__device__ __forceinline__ uint32_t max_e16x2(uint32_t w, uint32_t floor) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2_t, w),
                                                                __builtin_bit_cast(s16x2_t, floor)));
}

__device__ __forceinline__ void unpack4(const uint2& v, float* f) {
  f[0] = lo2f(v.x); f[1] = hi2f(v.x);
  f[2] = lo2f(v.y); f[3] = hi2f(v.y);
}

__device__ __forceinline__ uint2 pack4(const float* f) {
  return make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3]));
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5, "XCD swizzle must
// be bijective"): consecutive remapped ids land on the same XCD so neighbouring tiles share its L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  if (nwg < PVA_NXCD * 2) return orig;
  const int q = nwg / PVA_NXCD, r = nwg % PVA_NXCD;
  const int xcd = orig % PVA_NXCD;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / PVA_NXCD;
}


// v of the lane selected by DPP control CTRL (within each 16-lane row)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}

// Sum across the 16 lanes that share (lane >> 4), every lane getting the sum: four DPP-modified adds (quad_perm
// [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror) instead of __shfl_xor, which compiles to
// ds_bpermute_b32 — an LDS round trip and an lgkmcnt wait per step, 64 of them in a 16-value epilogue.
__device__ __forceinline__ float sum16(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return v;
}

// Sum across aligned groups of G adjacent lanes (G = 1, 2, 4, 8, 16), every lane getting its group's sum (DPP, as
// sum16: after the quad steps every lane of a quad holds the same value, so the mirrors pair whole quads / halves)
template <int G>
__device__ __forceinline__ float sum_lanes(float v) {
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "DPP lane groups stay inside a 16-lane row");
  if constexpr (G >= 2) v += dpp_f<0xB1>(v);
  if constexpr (G >= 4) v += dpp_f<0x4E>(v);
  if constexpr (G >= 8) v += dpp_f<0x141>(v);
  if constexpr (G >= 16) v += dpp_f<0x140>(v);
  return v;
}

// v[l] + v[l ^ 16] and v[l] + v[l ^ 32] for every lane: gfx950's row / half-wave swaps (v_permlane16_swap_b32 with
// vdst = src = v leaves rows (r0, r0, r2, r2) in one result and (r1, r1, r3, r3) in the other; likewise for halves;
// tools/probe/permlane_probe.hip).  fetch-inactive set: like ds_bpermute, a lane's partner is read even when the
// partner is outside EXEC.  The results are copied to scalars first (a bit_cast of the vector element r[1] reads
// element 0).
__device__ __forceinline__ float swap_sum16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), true, false);
  const unsigned a = r[0], b = r[1];
  return __uint_as_float(a) + __uint_as_float(b);
}
__device__ __forceinline__ float swap_sum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), true, false);
  const unsigned a = r[0], b = r[1];
  return __uint_as_float(a) + __uint_as_float(b);
}

// Sum over the lanes sharing (lane % S), S a compile-time power of two <= 64, every lane getting its group's sum:
// row_ror:4 / row_ror:8 DPP adds inside 16-lane rows, permlane swaps across rows (no ds_bpermute round trips).
// (quad_perm xor steps for strides 1 and 2).  Full-EXEC callers only: DPP does not read lanes outside EXEC.
template <int S>
__device__ __forceinline__ float wave_sum_stride_c(float v) {
  static_assert(S >= 1 && S <= 64 && (S & (S - 1)) == 0, "stride");
  if constexpr (S <= 1) v += dpp_f<0xB1>(v);
  if constexpr (S <= 2) v += dpp_f<0x4E>(v);
  if constexpr (S <= 4) v += dpp_f<0x124>(v);
  if constexpr (S <= 8) v += dpp_f<0x128>(v);
  if constexpr (S <= 16) v = swap_sum16(v);
  if constexpr (S <= 32) v = swap_sum32(v);
  return v;
}

// Sum over the whole wave (full EXEC), every lane getting it
__device__ __forceinline__ float wave_sum(float v) { return swap_sum32(swap_sum16(sum16(v))); }

// v of lane l ^ 16 (fetch-inactive, as ds_bpermute)
__device__ __forceinline__ unsigned swap_partner16(unsigned v) {
  const auto r = __builtin_amdgcn_permlane16_swap(v, v, true, false);
  const unsigned a = r[0], b = r[1];
  return a ^ b ^ v;
}

// Sum over the lanes of a wave that share (lane % S), S a power of two <= 64 (uniform).  Every lane
// gets its group's sum.  Used before LDS atomics: same-address ds_add_f32 lanes serialise badly.
__device__ __forceinline__ float wave_sum_stride(float v, int S) {
  switch (S) {   // (wave-uniform; full-EXEC callers)
    case 1: return wave_sum_stride_c<1>(v);
    case 2: return wave_sum_stride_c<2>(v);
    case 4: return wave_sum_stride_c<4>(v);
    case 8: return wave_sum_stride_c<8>(v);
    case 16: return wave_sum_stride_c<16>(v);
    case 32: return wave_sum_stride_c<32>(v);
    default:
      for (int off = S; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
      return v;
  }
}

// Sum across lanes l, l^16, l^32, l^48 (same lane & 15).
__device__ __forceinline__ float sum_hi4(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
