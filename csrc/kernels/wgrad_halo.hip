// Halo-staged weight gradient for stride-1 "same"-padded convolutions (gfx950): the 3x3 conv_b of every
// bottleneck and the temporal (3,1,1) conv_a of the fast pathway.
//
//   dW[n][k = (tap, cin)] = sum_p dY[p][n] * X[p + tap offset][cin]
//
// The tile kernel of conv_wgrad.hip gathers one im2col row per (position, tap): every input element is
// fetched once per tap, and at the 3x3 layers those re-reads miss L2 (profiles/r2_pmc_b64: 12.7 GB read per
// step at 9 % L2 hits for slow-res2 conv_b at B=64).  Here a workgroup walks BOXES of output positions (BT
// frames x BH rows x the full width); per box it stages dY [box positions][Cout] and the input HALO
// [(BT+kt-1) x (BH+kh-1) x (W+kw-1)][Cin] into LDS once, and every tap's operand is the same halo image read
// at a shifted row.  Fragments are read with the hardware-transpose LDS read (ds_read_b64_tr_b16: each lane
// supplies its own row address, so the per-tap shift and the box's row wrap are just per-lane row indices).
//   * 8 waves; WK waves split the block's k-tiles, WP waves split the 32-position chunks of a box; each wave
//     holds NTW (all) n-tiles x KTW k-tiles of 16x16 fp32 accumulators for its whole box range and adds them
//     into the zeroed fp32 accumulator with no-return atomics at the end (as conv_wgrad's split-K).
//   * Box staging goes global -> registers -> LDS through box-invariant row tables (no per-load division);
//     the next box's loads are issued before the current box's MFMAs (one barrier pair per box for the LDS
//     hand-over).  The producer's BN+ReLU is recomputed on the halo when it is stored (padding stays zero).
// Launch word (WgradParams::variant): bit 5 = this kernel; bits 8-11 BH, 12-14 BT, 15-16 log2 WP,
// 17-24 k-tiles per workgroup (k-tile groups x box splits, XCD-local); p_per_split = boxes per workgroup.
// (WP = 1, 4 or 8; NTW = 1, 2, 4 or 8 n-tiles of 16 = Cout rounded up.)
#include "common.h"
#include "conv_params.h"

PVA_NS_BEGIN

namespace {

constexpr int HX_THREADS = 512;
constexpr int HX_RA = 4, HX_RB = 6;   // 16-B staging registers per thread: <= 32 KB of dY, 48 KB of halo

__device__ __forceinline__ s16x4_t tr_read(const char* base) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(base));
}

// [rows][rowbytes] bf16 image of 32-byte segments, XOR-swizzled by row bits like conv_wgrad's img_off so the
// 8 rows a 32-lane half of a transpose read touches hit distinct bank groups (runtime row length)
__device__ __forceinline__ int himg(int row, int colbyte, int rowbytes) {
  const int nseg = rowbytes >> 5;
  int h = 0;
  if (nseg >= 8) h = (row & 3) | (((row >> 3) & 1) << 2);
  else if (nseg == 4) h = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  else if (nseg == 2) h = (row >> 3) & 1;
  return row * rowbytes + ((((colbyte >> 5) ^ h) << 5) | (colbyte & 31));
}

struct HaloGeo {
  int BT, BH, W, H, T, N;
  int HT, HH, HWd;   // halo extents
  int PB, PBp;       // box positions, padded to 32
  int HP;            // halo positions
  int coutp;         // dY image columns (Cout rounded up to 16)
  int nTB, nHB, nboxes;
};

__device__ __forceinline__ HaloGeo halo_geo(const WgradParams& p) {
  HaloGeo G;
  G.BH = (p.variant >> 8) & 15;
  G.BT = (p.variant >> 12) & 7;
  G.W = p.Wo; G.H = p.Ho; G.T = p.To;
  G.N = p.P / (G.T * G.H * G.W);
  G.HT = G.BT + p.kt - 1; G.HH = G.BH + p.kh - 1; G.HWd = G.W + p.kw - 1;
  G.PB = G.BT * G.BH * G.W;
  G.PBp = (G.PB + 31) & ~31;
  G.HP = G.HT * G.HH * G.HWd;
  G.coutp = (p.Cout + 15) & ~15;
  G.nTB = (G.T + G.BT - 1) / G.BT;
  G.nHB = (G.H + G.BH - 1) / G.BH;
  G.nboxes = G.N * G.nTB * G.nHB;
  return G;
}

template <int NTW, int KTW, int WP>
__global__ __launch_bounds__(HX_THREADS) void wgrad_halo_kernel(const WgradParams p) {
  constexpr int WK = 8 / WP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const HaloGeo G = halo_geo(p);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wk = wid % WK, wp = wid / WK;
  const int g = lane >> 4, li = lane & 15;
  const int rowA = G.coutp * 2, rowB = p.Cin * 2;
  char* A = smem;                                          // [PBp][coutp]
  char* B = smem + G.PBp * rowA;                           // [HP][Cin]
  int* htab = reinterpret_cast<int*>(B + G.HP * rowB);     // [PBp] halo row of each box position

  // box-invariant halo row of every box position (padding positions -> row 0; their dY rows are zero)
  for (int q = tid; q < G.PBp; q += HX_THREADS) {
    int v = 0;
    if (q < G.PB) {
      const int t = q / (G.BH * G.W), r = q - t * G.BH * G.W;
      const int h = r / G.W, w = r - h * G.W;
      v = (t * G.HH + h) * G.HWd + w;
    }
    htab[q] = v;
  }
  // this wave's k-tiles: per-lane (halo row offset of the tap, column byte) of the 4 columns it supplies
  const int KT = (p.K + 15) >> 4;
  const int ktb = (p.variant >> 17) & 255;
  // 1-D XCD-aware grid: the k-tile groups of one box range are neighbours on one XCD (its L2 serves them)
  const int ngroups = (KT + ktb - 1) / ktb;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int bsplit = lid / ngroups;
  const int kt0 = (lid - bsplit * ngroups) * ktb;
  const int kt_end = min(KT, kt0 + ktb);
  int ktoff[KTW], kcolb[KTW];
  bool kok[KTW];
#pragma unroll
  for (int j = 0; j < KTW; ++j) {
    const int kt = kt0 + wk * KTW + j;
    kok[j] = kt < kt_end;
    const int col = min(kt * 16 + 4 * (li & 3), p.K - 4);   // 4 columns, one tap (Cin % 4 == 0)
    const int tap = col / p.Cin, c = col - tap * p.Cin;
    const int dt = tap / (p.kh * p.kw), r = tap - dt * p.kh * p.kw;
    const int dh = r / p.kw, dw = r - dh * p.kw;
    ktoff[j] = (dt * G.HH + dh) * G.HWd + dw;
    kcolb[j] = c * 2;
  }
  f32x4_t acc[NTW][KTW];
#pragma unroll
  for (int i = 0; i < NTW; ++i)
#pragma unroll
    for (int j = 0; j < KTW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int cpa = G.coutp >> 3, cpb = p.Cin >> 3;   // 16-B chunks per dY / halo row (powers of two)
  const int la = 31 - __clz(cpa), lb = 31 - __clz(cpb);
  const int CHA = G.PBp * cpa, CH = CHA + G.HP * cpb;
  const int affine = p.affine;
  // box-invariant coordinates of every staged row, packed t | h << 4 | w << 14 (LDS tables)
  int* atab = htab + G.PBp;                                   // [PBp]  dY rows (t, h, w) in the box; -1 = pad
  int* btab = atab + G.PBp;                                   // [HP]   halo rows (t, h, w) relative to the box
  float* affs = reinterpret_cast<float*>(btab + G.HP);        // [2][Cin]
  for (int q = tid; q < G.PBp; q += HX_THREADS) {
    int v = -1;
    if (q < G.PB) {
      const int t = q / (G.BH * G.W), r = q - t * G.BH * G.W;
      const int h = r / G.W, w = r - h * G.W;
      v = t | (h << 4) | (w << 14);
    }
    atab[q] = v;
  }
  for (int q = tid; q < G.HP; q += HX_THREADS) {
    const int t = q / (G.HH * G.HWd), r = q - t * G.HH * G.HWd;
    const int h = r / G.HWd, w = r - h * G.HWd;
    btab[q] = t | (h << 4) | (w << 14);
  }
  if (affine)
    for (int i = tid; i < p.Cin; i += HX_THREADS) { affs[i] = p.in_scale[i]; affs[p.Cin + i] = p.in_shift[i]; }

  // box staging: global -> registers (issued before the previous box's MFMAs) -> LDS.  Raw buffer loads
  // with 32-bit offsets; padding / out-of-image chunks use an out-of-range offset and read zeros.
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, (short)0, (int)p.dybytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)p.xbytes, 0x00020000);
  constexpr unsigned OOB = 0xFFFFFFF0u;
  const int CHB = G.HP * cpb;
  uint4 sa[HX_RA], sb[HX_RB];
  unsigned vmask = 0;   // in-image halo chunks of the staged box: the affine applies to these only
  auto load = [&](int box) {
    int b = box;
    const int hb = b % G.nHB; b /= G.nHB;
    const int tb = b % G.nTB; const int n = b / G.nTB;
    const int t0 = tb * G.BT, h0 = hb * G.BH;
    const int nbase = n * G.T;
#pragma unroll
    for (int u = 0; u < HX_RA; ++u) {
      const int q = tid + u * HX_THREADS;
      const int row = q >> la, c8 = q & (cpa - 1);
      const int e = q < CHA ? atab[row] : -1;
      const int t = t0 + (e & 15), h = h0 + ((e >> 4) & 1023), w = e >> 14;
      const bool ok = e >= 0 && c8 * 8 < p.Cout && t < G.T && h < G.H;
      const int off = ((((nbase + t) * G.H + h) * G.W + w) * p.ldd + c8 * 8) * 2;
      sa[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(dyr, ok ? off : (int)OOB, 0, 0));
    }
    vmask = 0;
#pragma unroll
    for (int u = 0; u < HX_RB; ++u) {
      const int q = tid + u * HX_THREADS;
      const int row = q >> lb, c8 = q & (cpb - 1);
      const int e = q < CHB ? btab[row] : 0;
      const int ti = t0 + (e & 15) - p.pt, hi = h0 + ((e >> 4) & 1023) - p.ph, wi = (e >> 14) - p.pw;
      const bool ok = q < CHB && (unsigned)ti < (unsigned)G.T && (unsigned)hi < (unsigned)G.H &&
                      (unsigned)wi < (unsigned)G.W;
      const int off = ((((nbase + ti) * G.H + hi) * G.W + wi) * p.ldx + c8 * 8) * 2;
      sb[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? off : (int)OOB, 0, 0));
      vmask |= (unsigned)ok << u;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < HX_RA; ++u) {
      const int q = tid + u * HX_THREADS;
      if (q < CHA) *reinterpret_cast<uint4*>(A + himg(q >> la, (q & (cpa - 1)) * 16, rowA)) = sa[u];
    }
#pragma unroll
    for (int u = 0; u < HX_RB; ++u) {
      const int q = tid + u * HX_THREADS;
      if (q >= CHB) continue;
      const int c8 = q & (cpb - 1);
      uint4 v = sb[u];
      if (affine && ((vmask >> u) & 1u)) {   // BN(+ReLU) recompute of in-image chunks; padding stays zero
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float z = __builtin_fmaf(f[k], affs[c8 * 8 + k], affs[p.Cin + c8 * 8 + k]);
          f[k] = affine == 2 ? fmaxf(z, 0.f) : z;
        }
        v = pack8_fast(f);
      }
      *reinterpret_cast<uint4*>(B + himg(q >> lb, c8 * 16, rowB)) = v;
    }
  };

  const int box0 = bsplit * p.p_per_split;
  const int box1 = min(G.nboxes, box0 + p.p_per_split);
  const int nchunk = G.PBp >> 5;
  __syncthreads();   // tables
  if (box0 < box1) load(box0);
  for (int box = box0; box < box1; ++box) {
    __syncthreads();   // the previous box's fragments have been read
    store();
    __syncthreads();
    if (box + 1 < box1) load(box + 1);   // in flight under this box's MFMAs
    for (int ch = wp; ch < nchunk; ch += WP) {
      const int plo = ch * 32 + 8 * g + (li >> 2), phi = plo + 4;
      ev8_t af[NTW];
#pragma unroll
      for (int i = 0; i < NTW; ++i) {
        const int cb = (i * 16 + 4 * (li & 3)) * 2;
        const s16x4_t lo = tr_read(A + himg(plo, cb, rowA));
        const s16x4_t hi = tr_read(A + himg(phi, cb, rowA));
        af[i] = __builtin_bit_cast(ev8_t, (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
      }
      const int hlo = htab[plo], hhi = htab[phi];
#pragma unroll
      for (int j = 0; j < KTW; ++j) {
        if (!kok[j]) continue;   // wave-uniform
        const s16x4_t blo = tr_read(B + himg(hlo + ktoff[j], kcolb[j], rowB));
        const s16x4_t bhi = tr_read(B + himg(hhi + ktoff[j], kcolb[j], rowB));
        const ev8_t bf =
            __builtin_bit_cast(ev8_t, (s16x8_t){blo[0], blo[1], blo[2], blo[3], bhi[0], bhi[1], bhi[2], bhi[3]});
#pragma unroll
        for (int i = 0; i < NTW; ++i) acc[i][j] = PVA_MFMA16(af[i], bf, acc[i][j], 0, 0, 0);
      }
    }
  }
  // D[n][k]: lane holds k = kt*16 + li, n = i*16 + 4g + r
#pragma unroll
  for (int j = 0; j < KTW; ++j) {
    if (!kok[j]) continue;
    const int k = (kt0 + wk * KTW + j) * 16 + li;
#pragma unroll
    for (int i = 0; i < NTW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = i * 16 + 4 * g + r;
        if (n < p.Cout && k < p.K) atomicAdd(p.partial + (int64_t)n * p.K + k, acc[i][j][r]);
      }
  }
}

// KTW (k-tiles per wave) is rounded up to an instantiated width: surplus tiles fail the k-tile range test
template <int NTW, int WP>
void launch_k(const WgradParams& p, int ktw, dim3 grid, size_t lds, hipStream_t s) {
  if (ktw <= 2) hipLaunchKernelGGL((wgrad_halo_kernel<NTW, 2, WP>), grid, dim3(HX_THREADS), lds, s, p);
  else if (ktw == 3) hipLaunchKernelGGL((wgrad_halo_kernel<NTW, 3, WP>), grid, dim3(HX_THREADS), lds, s, p);
  else if (ktw == 4) hipLaunchKernelGGL((wgrad_halo_kernel<NTW, 4, WP>), grid, dim3(HX_THREADS), lds, s, p);
  else if constexpr (NTW <= 4) {
    if (ktw == 5) hipLaunchKernelGGL((wgrad_halo_kernel<NTW, 5, WP>), grid, dim3(HX_THREADS), lds, s, p);
    else if (ktw <= 6) hipLaunchKernelGGL((wgrad_halo_kernel<NTW, 6, WP>), grid, dim3(HX_THREADS), lds, s, p);
    else hipLaunchKernelGGL((wgrad_halo_kernel<NTW, 8, WP>), grid, dim3(HX_THREADS), lds, s, p);
  }
}

template <int NTW>
void launch_wp(const WgradParams& p, int wpl, int ktw, dim3 grid, size_t lds, hipStream_t s) {
  switch (wpl) {
    case 0: launch_k<NTW, 1>(p, ktw, grid, lds, s); break;
    case 2: launch_k<NTW, 4>(p, ktw, grid, lds, s); break;
    default: launch_k<NTW, 8>(p, ktw, grid, lds, s); break;
  }
}

struct HostGeo {
  int PB, PBp, HP, coutp, nboxes, KT, ktb, ktw, ntw, wpl, chunks;
  size_t lds;
};

HostGeo host_geo(const WgradParams& p) {
  HostGeo h;
  const int BH = (p.variant >> 8) & 15, BT = (p.variant >> 12) & 7;
  h.wpl = (p.variant >> 15) & 3;
  h.ktb = (p.variant >> 17) & 255;
  h.PB = BT * BH * p.Wo;
  h.PBp = (h.PB + 31) & ~31;
  h.HP = (BT + p.kt - 1) * (BH + p.kh - 1) * (p.Wo + p.kw - 1);
  h.coutp = (p.Cout + 15) & ~15;
  const int N = p.P / (p.To * p.Ho * p.Wo);
  h.nboxes = N * ((p.To + BT - 1) / BT) * ((p.Ho + BH - 1) / BH);
  h.KT = (p.K + 15) / 16;
  const int WK = 8 >> h.wpl;
  h.ktw = (h.ktb + WK - 1) / WK;
  h.ntw = h.coutp / 16;
  h.chunks = h.PBp * (h.coutp / 8) + h.HP * (p.Cin / 8);
  h.lds = (size_t)h.PBp * h.coutp * 2 + (size_t)h.HP * p.Cin * 2 + (size_t)(2 * h.PBp + h.HP) * 4 +
          (p.affine ? (size_t)p.Cin * 8 : 0);
  return h;
}

}  // namespace

// 1 when the halo kernel can run this weight gradient with launch word `variant`
int wgrad_halo_legal(const WgradParams& p) {
  if (p.variant < 0 || !(p.variant & 32)) return 0;
  if (p.st != 1 || p.sh != 1 || p.sw != 1) return 0;
  if (p.Ti != p.To || p.Hi != p.Ho || p.Wi != p.Wo) return 0;
  if (p.pt != (p.kt - 1) / 2 || p.ph != (p.kh - 1) / 2 || p.pw != (p.kw - 1) / 2) return 0;
  if (p.Cin % 8 != 0 || p.Cout > 128 || p.slab || p.dy_affine) return 0;
  if (p.ldd % 8 != 0 || p.ldx % 8 != 0) return 0;
  if (p.P % (p.To * p.Ho * p.Wo) != 0) return 0;
  const int BH = (p.variant >> 8) & 15, BT = (p.variant >> 12) & 7;
  if (BH < 1 || BT < 1) return 0;
  const HostGeo h = host_geo(p);
  if (h.wpl == 1) return 0;   // waves per position chunk: 1, 4 or 8
  const int ktw_inst = h.ktw <= 2 ? 2 : h.ktw <= 5 ? h.ktw : h.ktw <= 6 ? 6 : 8;
  if (h.ktb < 1 || h.ktw > 8 || h.ntw > 8 || h.ntw == 3 || (h.ntw > 4 && h.ntw < 8) || h.ntw * ktw_inst > 32)
    return 0;
  if (h.lds > 150 * 1024 || h.PBp * (h.coutp / 8) > HX_RA * HX_THREADS || h.HP * (p.Cin / 8) > HX_RB * HX_THREADS || (p.Cin & (p.Cin - 1)) || p.Wo >= 1024 || p.Ho >= 1024)
    return 0;
  return 1;
}

void wgrad_halo_launch(const WgradParams& p, hipStream_t s) {
  const HostGeo h = host_geo(p);
  const int splits = (h.nboxes + p.p_per_split - 1) / p.p_per_split;
  const dim3 grid(splits * ((h.KT + h.ktb - 1) / h.ktb));
  switch (h.ntw) {
    case 1: launch_wp<1>(p, h.wpl, h.ktw, grid, h.lds, s); break;
    case 2: launch_wp<2>(p, h.wpl, h.ktw, grid, h.lds, s); break;
    case 4: launch_wp<4>(p, h.wpl, h.ktw, grid, h.lds, s); break;
    default: launch_wp<8>(p, h.wpl, h.ktw, grid, h.lds, s); break;
  }
}

PVA_NS_END  // namespace PVA_NS
