// Optimizer step, bf16 weight packing and on-device video preprocessing (gfx950).
//
// * sgd_momentum_kernel: one launch over the flat fp32 master buffer (all 330+ parameter tensors):
//   g' = g*gscale + wd*p ; buf = first ? g' : m*buf + g' ; p -= lr*buf  (torch.optim.SGD semantics,
//   dampening 0, no nesterov).  lr is read from device memory so a captured HIP graph
//   replays with the live cosine schedule value.  Non-finite gradients raise a device flag (fp16 scaler).
// * pack_weights_kernel: multi-tensor fp32 [Cout][Cin][kt][kh][kw] -> bf16 packed forward layout
//   [Cout][taps][Cin_pad] and dgrad layout [Cin][taps][Cout] in one launch (gridDim.y = tensor).
// * video_preprocess_kernel: uint8 THWC decoded frames -> normalised bf16 NDHWC RGB0 clip: temporal
//   index gather (UniformTemporalSubsample / PackPathway), bilinear short-side resize (align_corners =
//   False, PyTorch source-index rule), crop, horizontal flip, (x/255 - mean)/std, all in one pass
//   (normalisation commutes with the bilinear resize since the weights sum to 1).
#include "common.h"

PVA_NS_BEGIN

namespace {

// GradScaler pre-pass: flag = 1 if any g*gscale is inf/nan (torch _amp_foreach_non_finite_check_and_unscale_)
__global__ void nonfinite_check_kernel(const float* __restrict__ g, int64_t n, float gscale, int* __restrict__ flag) {
  bool bad = false;
  const int64_t n4 = n >> 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(g)[i];
    bad |= !isfinite(v.x * gscale) || !isfinite(v.y * gscale) || !isfinite(v.z * gscale) || !isfinite(v.w * gscale);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) bad |= !isfinite(g[(n4 << 2) + threadIdx.x] * gscale);
  if (__any(bad) && (threadIdx.x & 63) == 0) *flag = 1;   // benign race: every writer stores 1
}

__global__ void sgd_momentum_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf,
                                    int64_t n, const float* __restrict__ lr_ptr, float momentum, float wd,
                                    float gscale, int first, int* __restrict__ found_inf,
                                    const int* __restrict__ skip_flag) {
  if (skip_flag && *skip_flag) return;   // overflowed fp16-scaled step: parameters and momentum untouched
  const float lr = *lr_ptr;
  const int64_t n4 = n >> 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 bv = first ? float4{0, 0, 0, 0} : reinterpret_cast<float4*>(buf)[i];
    float* pp = &pv.x; float* gg = &gv.x; float* bb = &bv.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float gr = gg[e] * gscale;
      if (found_inf && !isfinite(gr)) *found_inf = 1;
      gr += wd * pp[e];
      bb[e] = first ? gr : momentum * bb[e] + gr;
      pp[e] -= lr * bb[e];
    }
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(buf)[i] = bv;
  }
  // tail
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = (n4 << 2) + threadIdx.x;
    float gr = g[i] * gscale;
    if (found_inf && !isfinite(gr)) *found_inf = 1;
    gr += wd * p[i];
    buf[i] = first ? gr : momentum * buf[i] + gr;
    p[i] -= lr * buf[i];
  }
}

struct PackDesc {
  int64_t src;     // offset in fp32 master buffer
  int64_t fwd;     // offset in bf16 forward-pack buffer
  int64_t dgr;     // offset in bf16 dgrad-pack buffer (-1: none)
  int cout, cin, cin_pad, taps;
};

// One 32(cout) x 32(cin) tile of one tap per block iteration, staged through LDS: the forward layout
// [Cout][taps][Cin_pad] is written along cin, the dgrad layout [Cin][taps][Cout] along cout, so both
// stores are contiguous (the dgrad pack is a transpose; scattered 2-B stores made it 10x slower).
__global__ void pack_weights_kernel(const float* __restrict__ master, uint16_t* __restrict__ fwd,
                                    uint16_t* __restrict__ dgr, const PackDesc* __restrict__ descs) {
  const PackDesc d = descs[blockIdx.y];
  const float* src = master + d.src;
  uint16_t* fo = fwd + d.fwd;
  uint16_t* dg = d.dgr >= 0 ? dgr + d.dgr : nullptr;
  __shared__ uint16_t tile[32][33];
  const int tn = (d.cout + 31) / 32, tc = (d.cin + 31) / 32;
  const int ntiles = tn * tc * d.taps;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tap = t % d.taps;
    const int r = t / d.taps;
    const int cb = (r % tc) * 32, nb = (r / tc) * 32;
    // load rows n, columns c (source stride taps along c)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int n = nb + ty + 8 * k, c = cb + tx;
      uint16_t v = 0;
      if (n < d.cout && c < d.cin) {
        v = f2e(src[(n * d.cin + c) * d.taps + tap]);
        fo[(n * d.taps + tap) * d.cin_pad + c] = v;
      }
      tile[ty + 8 * k][tx] = v;
    }
    if (dg) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = cb + ty + 8 * k, n = nb + tx;
        if (n < d.cout && c < d.cin) dg[(c * d.taps + tap) * d.cout + n] = tile[tx][ty + 8 * k];
      }
    }
    __syncthreads();
  }
}

// frames: packed uint8 clips, clip b = [Ts][Hs][Ws][3] at byte offset desc[b].off ;
// desc: [B][10] int32 = (off_lo, off_hi, Ts, Hs, Ws, rh, rw, top, left, flip) ; tidx: [B][T] frame index
// inside the clip ; out: [B][T][S][S][4] bf16 (channel 3 = 0), or s2d [B][T][S/2][S/2][16].  Per-clip geometry lets
// one launch serve a batch of differently sized source videos.  Each thread produces a 2x2 output cell (s2d: one 32-B,
// 16-channel position — two 16-B stores, consecutive threads consecutive cells; NDHWC RGB0: 16 B per output row); the
// per-pixel arithmetic is the original per-pixel kernel's, expression for expression (bitwise the same values).
// Measured (profiles/r4_pmc): the per-pixel form took 2.7 ms/step at B=160 — 12 byte loads and an 8-B store per pixel
// with half-filled 32-B sectors in the s2d layout.

__device__ __forceinline__ void pre_pixel(const uint8_t* f, int Ws, int x0, int x1, float lx, int y0r, int y1r, float ly,
                                          float m0, float m1, float m2, float is0, float is1, float is2, float* v) {
  const uint8_t* p00 = f + (y0r * Ws + x0) * 3;
  const uint8_t* p01 = f + (y0r * Ws + x1) * 3;
  const uint8_t* p10 = f + (y1r * Ws + x0) * 3;
  const uint8_t* p11 = f + (y1r * Ws + x1) * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float top_ = (1.f - lx) * (float)p00[c] + lx * (float)p01[c];
    const float bot_ = (1.f - lx) * (float)p10[c] + lx * (float)p11[c];
    v[c] = (1.f - ly) * top_ + ly * bot_;
  }
  v[0] = (v[0] * (1.f / 255.f) - m0) * is0;
  v[1] = (v[1] * (1.f / 255.f) - m1) * is1;
  v[2] = (v[2] * (1.f / 255.f) - m2) * is2;
  v[3] = 0.f;
}

// A workgroup owns PRE2_RP output row pairs of one frame.  The previous row-pair form (one workgroup per 2 output
// rows, profiles/r5_preprocess) paid a dependent chain per 2 output rows — descriptor, frame index, then the rows
// (three memory latencies, ~13 us per unit measured: 1.1 TB/s, scripts/preprocess_bench.py); here the descriptor
// and frame index are read once, the whole source-row span of the chunk is copied to LDS by LDS-DMA in one phase
// (4-B lanes, no VGPR staging), and 256 threads then produce the chunk's cells.  Same per-pixel arithmetic.
constexpr int PRE2_RP = 8, PRE2_LDS = 24 * 1024;

__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t r, uint8_t* lds, int voff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 4, voff, 0, 0, 0);
#endif
}

__global__ __launch_bounds__(256) void video_preprocess2_kernel(const uint8_t* __restrict__ frames,
                                                                const int* __restrict__ desc,
                                                                const int* __restrict__ tidx, int T, int S, float m0,
                                                                float m1, float m2, float is0, float is1, float is2,
                                                                uint16_t* __restrict__ out, int s2d,
                                                                const int* __restrict__ slow_of,
                                                                uint16_t* __restrict__ slow_out, int Ts) {
  __shared__ __attribute__((aligned(16))) uint8_t rows[PRE2_LDS];
  const int RP = (S + 1) >> 1;
  const int nch = (RP + PRE2_RP - 1) / PRE2_RP;
  const int u = blockIdx.x;
  const int b = u / (T * nch);
  const int rem = u - b * T * nch;
  const int t = rem / nch, ch = rem - t * nch;
  const int* d = desc + b * 10;
  const int64_t off = (int64_t)(uint32_t)d[0] | ((int64_t)d[1] << 31);
  const int Hs = d[3], Ws = d[4], rh = d[5], rw = d[6], top = d[7], left = d[8], flip = d[9];
  const uint8_t* f = frames + off + (int64_t)tidx[b * T + t] * Hs * Ws * 3;
  const int r0 = ch * PRE2_RP, r1 = min(RP, r0 + PRE2_RP);
  // slow pathway: its frames are a subset of this clip's (pack_pathway_indices); frame t's cells also go to slow frame
  // slow_of[t] (-1: not a slow frame) — one pass over the source instead of a second launch
  const int ts = slow_out ? slow_of[t] : -1;
  auto src_rows = [&](int y, int& y0, int& y1, float& ly) {   // the row-pair form's expressions
    const float sy = fmaxf(((float)(y + top) + 0.5f) * ((float)Hs / (float)rh) - 0.5f, 0.f);
    y0 = min((int)sy, Hs - 1);
    y1 = min(y0 + 1, Hs - 1);
    ly = sy - (float)y0;
  };
  int ylo, yhi, dummy;
  float fd;
  src_rows(2 * r0, ylo, dummy, fd);
  src_rows(min(2 * r1 - 1, S - 1), dummy, yhi, fd);
  const int rowb = Ws * 3;
  const int span = (yhi - ylo + 1) * rowb;
  const uint8_t* src = f + (int64_t)ylo * rowb;
  const bool staged = span <= PRE2_LDS && (((uintptr_t)src | (uintptr_t)span) & 3) == 0;
  if (staged) {
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, span, 0x00020000);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nchunk = (span + 255) >> 8;   // 256-B wave chunks (lanes past the span read zeros)
    for (int k = w; k < nchunk; k += 4) dma4(sr, rows + k * 256, k * 256 + lane * 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  auto cells = [&](const uint8_t* base) {
    const int ncell = (r1 - r0) * RP;
    for (int q = threadIdx.x; q < ncell; q += 256) {
      const int r = r0 + q / RP, c = q - (q / RP) * RP;
      int y0s[2], y1s[2];
      float lys[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) src_rows(min(2 * r + k, S - 1), y0s[k], y1s[k], lys[k]);
      float v[2][2][4];
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int x = min(2 * c + dx, S - 1);
        const int xr = (flip ? (S - 1 - x) : x) + left;
        const float sx = fmaxf(((float)xr + 0.5f) * ((float)Ws / (float)rw) - 0.5f, 0.f);
        const int x0 = min((int)sx, Ws - 1);
        const int x1 = min(x0 + 1, Ws - 1);
        const float lx = sx - (float)x0;
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
          pre_pixel(base, Ws, x0, x1, lx, y0s[dy] - ylo, y1s[dy] - ylo, lys[dy], m0, m1, m2, is0, is1, is2, v[dy][dx]);
      }
      const uint2 q00 = pack4(v[0][0]), q01 = pack4(v[0][1]), q10 = pack4(v[1][0]), q11 = pack4(v[1][1]);
      auto store = [&](uint16_t* dst, int64_t fr) {
        if (s2d) {
          uint16_t* o = dst + ((fr * RP + r) * RP + c) * 16;
          *reinterpret_cast<uint4*>(o) = make_uint4(q00.x, q00.y, q01.x, q01.y);
          *reinterpret_cast<uint4*>(o + 8) = make_uint4(q10.x, q10.y, q11.x, q11.y);
        } else {
          const int y = 2 * r, x = 2 * c;
          uint16_t* o0 = dst + ((fr * S + y) * S + x) * 4;
          if (x + 1 < S) *reinterpret_cast<uint4*>(o0) = make_uint4(q00.x, q00.y, q01.x, q01.y);
          else *reinterpret_cast<uint2*>(o0) = q00;
          if (y + 1 < S) {
            uint16_t* o1 = o0 + (int64_t)S * 4;
            if (x + 1 < S) *reinterpret_cast<uint4*>(o1) = make_uint4(q10.x, q10.y, q11.x, q11.y);
            else *reinterpret_cast<uint2*>(o1) = q10;
          }
        }
      };
      store(out, (int64_t)b * T + t);
      if (ts >= 0) store(slow_out, (int64_t)b * Ts + ts);
    }
  };
  if (staged) cells(rows);
  else cells(src);
}

// synthetic decoded frames on device: deterministic hash -> uint8 (no zeros: DVFS, BASELINE.md protocol)
__global__ void synth_frames_kernel(uint8_t* __restrict__ out, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
    out[i] = (uint8_t)h;
  }
}

}  // namespace

void sgd_momentum_launch(float* p, const float* g, float* buf, int64_t n, const float* lr, float momentum, float wd,
                         float gscale, int first, int* found_inf, const int* skip_flag, hipStream_t s) {
  int64_t blocks = ((n >> 2) + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(sgd_momentum_kernel, dim3((int)blocks), dim3(256), 0, s, p, g, buf, n, lr, momentum, wd, gscale,
                     first, found_inf, skip_flag);
}

void nonfinite_check_launch(const float* g, int64_t n, float gscale, int* flag, hipStream_t s) {
  int64_t blocks = ((n >> 2) + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(nonfinite_check_kernel, dim3((int)blocks), dim3(256), 0, s, g, n, gscale, flag);
}

void pack_weights_launch(const float* master, uint16_t* fwd, uint16_t* dgr, const void* descs, int ntensors,
                         hipStream_t s) {
  hipLaunchKernelGGL(pack_weights_kernel, dim3(128, ntensors), dim3(256), 0, s, master, fwd, dgr,
                     reinterpret_cast<const PackDesc*>(descs));
}

int pack_desc_size() { return (int)sizeof(PackDesc); }

void video_preprocess_launch(const uint8_t* frames, const int* desc, const int* tidx, int B, int T, int S,
                             const float* mean, const float* std_, uint16_t* out, int s2d, hipStream_t s,
                             const int* slow_of, uint16_t* slow_out, int Ts) {
  const int RP = (S + 1) / 2;
  const int64_t wgs = (int64_t)B * T * ((RP + PRE2_RP - 1) / PRE2_RP);
  if (wgs <= 0) return;
  hipLaunchKernelGGL(video_preprocess2_kernel, dim3((unsigned)wgs), dim3(256), 0, s, frames, desc, tidx, T, S, mean[0],
                     mean[1], mean[2], 1.f / std_[0], 1.f / std_[1], 1.f / std_[2], out, s2d, slow_of, slow_out, Ts);
}

void synth_frames_launch(uint8_t* out, int64_t n, uint32_t seed, hipStream_t s) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(synth_frames_kernel, dim3((int)blocks), dim3(256), 0, s, out, n, seed);
}

PVA_NS_END  // namespace PVA_NS
