// pybind11 bindings of the gfx950 kernels (module pytorchvideo_accelerate_amd._C).
//
// Thin, allocation-free launch shims: every output buffer is pre-allocated by the Python executor
// (so a whole training step can be captured into a HIP graph), kernels run on PyTorch's current HIP
// stream, and shapes arrive as plain ints from the executor's static plan.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include "../kernels/conv_params.h"
#include <cstddef>

static_assert(offsetof(ConvParams, bws) - offsetof(ConvParams, M) == 38 * sizeof(int),
              "ConvParams integer block must be contiguous (filled from a 39-int geometry vector)");

// ---- kernel launchers (csrc/kernels/launchers.h), one set per 16-bit compute type ----
namespace pva_bf16 {
#include "../kernels/launchers.h"
}
namespace pva_f16 {
#include "../kernels/launchers.h"
}
void register_clip_reader(pybind11::module& m);
void register_rccl(pybind11::module& m);
void register_fp32(pybind11::module& m);

namespace {

using OptT = c10::optional<at::Tensor>;

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

// 16-bit compute type of the current call: set from the call's primary 16-bit tensor (kind16); every other 16-bit
// tensor of the call must match it.  bf16 tensors run the pva_bf16 kernels, fp16 tensors the pva_f16 kernels.
thread_local at::ScalarType tl_kind = at::kBFloat16;
inline bool kind16(const at::Tensor& t) {
  const auto k = t.scalar_type();
  TORCH_CHECK(k == at::kBFloat16 || k == at::kHalf, "expected a bf16 or fp16 tensor");
  tl_kind = k;
  return k == at::kHalf;
}
#define KSEL(h, fn) ((h) ? pva_f16::fn : pva_bf16::fn)

inline void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous() || t.dim() <= 2, name, " must be contiguous");
}
inline const uint16_t* bfp(const at::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == tl_kind, "expected a ", c10::toString(tl_kind), " tensor (one compute dtype per call)");
  return reinterpret_cast<const uint16_t*>(t.data_ptr());
}
inline uint16_t* bfpm(const at::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == tl_kind, "expected a ", c10::toString(tl_kind), " tensor (one compute dtype per call)");
  return reinterpret_cast<uint16_t*>(t.data_ptr());
}
inline const uint16_t* bfo(const OptT& t) { return t.has_value() ? bfp(*t) : nullptr; }
inline uint16_t* bfom(const OptT& t) { return t.has_value() ? bfpm(*t) : nullptr; }
inline float* f32(const at::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kFloat, "expected fp32 tensor");
  return t.data_ptr<float>();
}
inline float* f32o(const OptT& t) { return t.has_value() ? f32(*t) : nullptr; }

// geometry vector (39): [M, Ngemm, Kfull, Cg, ldx, ldy, Gt, Gh, Gw, Rt, Rh, Rw, Ot, Oh, Ow,
//   ost, osh, osw, ort, orh, orw, ast, ash, asw, aot, aoh, aow, dir, nt, nh, nw, kh, kw,
//   bt0, bh0, bw0, bts, bhs, bws]   (see ConvParams; built by ops/conv.py)
static ConvParams conv_params(const at::Tensor& x, const at::Tensor& w, const at::Tensor& y, int64_t accum,
                              const std::vector<int64_t>& g, int64_t chunk) {
  TORCH_CHECK(g.size() == 39, "conv geometry must have 39 entries");
  ConvParams p{};
  p.x = bfp(x); p.w = bfp(w); p.y = bfpm(y);
  p.accum = (int)accum;
  int* f = &p.M;
  for (int i = 0; i < 39; ++i) f[i] = (int)g[i];
  // bounds tests are only needed when some tap can read outside the gathered tensor
  auto dim_ok = [](int R, int as, int ao, int dir, int n, int G) {
    const int lo = ao + (dir < 0 ? -(n - 1) : 0);
    const int hi = (R - 1) * as + ao + (dir > 0 ? (n - 1) : 0);
    return n == 0 || (lo >= 0 && hi < G);
  };
  p.check = (dim_ok(p.Rt, p.ast, p.aot, p.dir, p.nt, p.Gt) && dim_ok(p.Rh, p.ash, p.aoh, p.dir, p.nh, p.Gh) &&
             dim_ok(p.Rw, p.asw, p.aow, p.dir, p.nw, p.Gw)) ? 0 : 1;
  TORCH_CHECK(x.numel() < (1ll << 31) && y.numel() < (1ll << 31), "tensor too large for 32-bit offsets");
  TORCH_CHECK(x.numel() * 2 < 0xFFFFFF00ll && w.numel() * 2 < 0xFFFFFF00ll, "buffer extents must fit 32 bits");
  p.xbytes = (unsigned)(x.numel() * 2);
  p.wbytes = (unsigned)(w.numel() * 2);
  TORCH_CHECK(p.Cg % chunk == 0 && p.Cg > 0, "gathered channels must be a multiple of the chunk");
  TORCH_CHECK(p.Ngemm % 4 == 0, "output channels must be a multiple of 4");
  TORCH_CHECK(p.ldx % chunk == 0 && p.ldy % 4 == 0, "row strides must keep vector alignment");
  TORCH_CHECK(w.numel() >= (int64_t)p.Ngemm * p.Kfull, "packed weight too small");
  return p;
}

// the streaming pointwise kernel (cfg bit 9) must only get geometries it supports: its slab count and row
// mapping differ from the tile kernels', so a silent fallback would corrupt the caller's partial sums
static void check_pw(const ConvParams& p, int64_t chunk, int64_t cfg) {
  if (cfg >= 0 && (cfg & 16) && (cfg & 2048)) {   // halo-staged 3x3 kernel: geometry, epilogue, tile size
    const int P = pva_bf16::conv_halo_legal(p, (int)chunk);
    TORCH_CHECK(P > 0 && P == (int)(cfg >> 12), "halo conv kernel selected for an unsupported geometry");
    TORCH_CHECK(pva_bf16::conv_halo_epi_ok(p), "halo conv kernel selected for an unsupported epilogue");
    TORCH_CHECK(!(cfg & 2) || pva_bf16::conv_halo64p_legal(p, (int)chunk) >= ((cfg & 8) ? 2 : 1),
                "persistent 64-channel halo conv kernel selected for an unsupported geometry");
    return;
  }
  if (cfg < 0 || !(cfg & 16) || !(cfg & 512)) return;
  TORCH_CHECK(pva_bf16::conv_pw_legal(p, (int)chunk), "pointwise conv kernel selected for an unsupported geometry");
  TORCH_CHECK(p.nt == 1 || p.xbytes < 0x80000000u, "temporal pointwise conv: input must stay under 2 GiB");
  TORCH_CHECK(!p.eres || p.ldr % 8 == 0, "pointwise conv kernel: residual row stride must be a multiple of 8");
  TORCH_CHECK(!p.emask || p.Ngemm % 8 == 0, "pointwise conv kernel: mask layout");
}

void conv_igemm(const at::Tensor& x, const at::Tensor& w, const at::Tensor& y, const OptT& stats,
                const OptT& scale, const OptT& shift, int64_t affine, int64_t accum, std::vector<int64_t> g,
                int64_t chunk, int64_t cfg, const OptT& bias, int64_t nostore) {
  const bool h = kind16(x);
  ConvParams p = conv_params(x, w, y, accum, g, chunk);
  p.nostore = (int)nostore;
  TORCH_CHECK(!nostore || (stats.has_value() && !accum && !bias.has_value()),
              "statistics-only forward needs stats and no accumulate / bias");
  p.ebias = f32o(bias);
  TORCH_CHECK(!bias.has_value() || bias->numel() >= p.Ngemm, "bias too small");
  p.stats = f32o(stats);
  p.in_scale = f32o(scale); p.in_shift = f32o(shift);
  p.affine = (int)affine;
  TORCH_CHECK(!affine || (scale.has_value() && shift.has_value()), "affine needs scale/shift");
  check_pw(p, chunk, cfg);
  if (p.M == 0) return;
  KSEL(h, conv_igemm_launch)(p, (int)chunk, cur_stream(), (int)cfg);
}

// forward conv whose epilogue applies its own BatchNorm from known statistics and writes the residual-unit
// output: out = relu(acc * fsc + fsh + r), r = res (identity) or res * rsc + rsh (branch1 BN); ReLU bits
// into mask [rows][Ngemm/8]
void conv_igemm_fres(const at::Tensor& x, const at::Tensor& w, const at::Tensor& y, const OptT& scale,
                     const OptT& shift, int64_t affine, std::vector<int64_t> g, int64_t chunk, int64_t cfg,
                     const at::Tensor& osc, const at::Tensor& osh, const at::Tensor& res, int64_t ldr,
                     const OptT& rsc, const OptT& rsh, const at::Tensor& mask) {
  const bool h = kind16(x);
  ConvParams p = conv_params(x, w, y, 0, g, chunk);
  TORCH_CHECK(chunk == 8, "fres epilogue needs 16-B chunks");
  p.in_scale = f32o(scale); p.in_shift = f32o(shift);
  p.affine = (int)affine;
  TORCH_CHECK(!affine || (scale.has_value() && shift.has_value()), "affine needs scale/shift");
  p.fres = 1;
  p.fsc = f32(osc); p.fsh = f32(osh);
  TORCH_CHECK(osc.numel() >= p.Ngemm && osh.numel() >= p.Ngemm, "output affine too small");
  p.eres = bfp(res); p.ldr = (int)ldr;
  TORCH_CHECK(ldr % 4 == 0, "residual row stride alignment");
  TORCH_CHECK(rsc.has_value() == rsh.has_value(), "residual affine needs scale and shift");
  p.rsc = f32o(rsc); p.rsh = f32o(rsh);
  TORCH_CHECK(mask.scalar_type() == at::kByte && p.Ngemm % 8 == 0 && mask.numel() >= (int64_t)p.M * (p.Ngemm / 8),
              "mask must be uint8 bits [rows][C/8]");
  p.emask_out = mask.data_ptr<uint8_t>();
  TORCH_CHECK(p.ost == 1 && p.osh == 1 && p.osw == 1, "fres epilogue: dense output rows");
  check_pw(p, chunk, cfg);
  if (p.M == 0) return;
  KSEL(h, conv_igemm_launch)(p, (int)chunk, cur_stream(), (int)cfg);
}

// dgrad with the backward-BN epilogue (see ConvParams): residual add, ReLU-bit mask, and partial sums
// [m_tiles][3][Ngemm] of (v, v*xhat0, v*xhat1) over this launch's rows (which must be dense: one phase).
void conv_igemm_epi(const at::Tensor& x, const at::Tensor& w, const at::Tensor& y, int64_t accum,
                    std::vector<int64_t> g, int64_t chunk, const OptT& res, int64_t ldr, const OptT& mask,
                    const OptT& y0, const OptT& mean0, const OptT& rstd0, const OptT& y1, const OptT& mean1,
                    const OptT& rstd1, const OptT& part, const OptT& msc, const OptT& msh, int64_t cfg,
                    const OptT& bias) {
  const bool h = kind16(x);
  ConvParams p = conv_params(x, w, y, accum, g, chunk);
  p.ebias = f32o(bias);
  TORCH_CHECK(!bias.has_value() || bias->numel() >= p.Ngemm, "bias too small");
  TORCH_CHECK(!bias.has_value() || cfg < 0 || !(cfg & 32), "the direct kernel has no bias epilogue");
  p.eres = bfo(res); p.ldr = (int)ldr;
  TORCH_CHECK(!res.has_value() || ldr % 4 == 0, "residual row stride alignment");
  if (mask.has_value()) {
    TORCH_CHECK(mask->scalar_type() == at::kByte && p.Ngemm % 8 == 0, "mask must be uint8 bits [rows][C/8]");
    p.emask = mask->data_ptr<uint8_t>();
  }
  if (part.has_value()) {
    TORCH_CHECK(!y0.has_value() || (mean0.has_value() && rstd0.has_value()), "BN epilogue needs mean0/rstd0 with y0");
    TORCH_CHECK(!(msc.has_value() && !y0.has_value()), "mask affine reads y0");
    TORCH_CHECK(!y1.has_value() || (mean1.has_value() && rstd1.has_value()), "BN epilogue needs mean1/rstd1");
    TORCH_CHECK(!y0.has_value() || y0->size(-1) == p.Ngemm, "BN epilogue inputs must be dense [rows][Ngemm]");
    p.ey0 = bfo(y0); p.ey1 = bfo(y1);
    p.emean0 = f32o(mean0); p.erstd0 = f32o(rstd0); p.emean1 = f32o(mean1); p.erstd1 = f32o(rstd1);
    p.epart = f32(*part);
    TORCH_CHECK(msc.has_value() == msh.has_value(), "mask affine needs scale and shift");
    p.emsc = f32o(msc); p.emsh = f32o(msh);
    const int bm = KSEL(h, conv_cfg_bm)((int)cfg, p.Ngemm);
    TORCH_CHECK(part->numel() >= (int64_t)((p.M + bm - 1) / bm) * 3 * p.Ngemm, "partials too small");
  }
  check_pw(p, chunk, cfg);
  if (p.M == 0) return;
  KSEL(h, conv_igemm_launch)(p, (int)chunk, cur_stream(), (int)cfg);
}

// row tiles of the BN partial-sum buffer a conv launch writes; pass K (= taps * Cg) and Cg for forward
// launches so the small-channel streaming kernel's 128-row tiles are accounted for
int64_t conv_m_tiles(int64_t M, int64_t N, int64_t K, int64_t Cg) {
  return K > 0 ? pva_bf16::conv_igemm_m_tiles_k((int)M, (int)N, (int)K, (int)Cg) : pva_bf16::conv_igemm_m_tiles((int)M, (int)N);
}

std::vector<int64_t> wgrad_tile(int64_t Cout, int64_t K, int64_t variant) {
  int a, b;
  pva_bf16::conv_wgrad_tile((int)Cout, (int)K, (int)variant, &a, &b);
  return {a, b};
}

// geometry: [P, Cout, K, Cin, ldd, ldx, Ti, Hi, Wi, To, Ho, Wo, kt, kh, kw, st, sh, sw, pt, ph, pw, splits, pps]
void conv_wgrad(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& partial, const OptT& scale,
                const OptT& shift, int64_t affine, std::vector<int64_t> g, int64_t chunk, int64_t slab,
                int64_t variant, int64_t dy_affine, const OptT& colsum) {
  const bool h = kind16(dy);
  TORCH_CHECK(g.size() == 23, "wgrad geometry must have 23 entries");
  WgradParams p{};
  p.dy = bfp(dy); p.x = bfp(x); p.partial = f32(partial);
  p.in_scale = f32o(scale); p.in_shift = f32o(shift); p.affine = (int)affine;
  p.P = g[0]; p.Cout = g[1]; p.K = g[2]; p.Cin = g[3]; p.ldd = g[4]; p.ldx = g[5];
  p.Ti = g[6]; p.Hi = g[7]; p.Wi = g[8]; p.To = g[9]; p.Ho = g[10]; p.Wo = g[11];
  p.kt = g[12]; p.kh = g[13]; p.kw = g[14]; p.st = g[15]; p.sh = g[16]; p.sw = g[17];
  p.pt = g[18]; p.ph = g[19]; p.pw = g[20]; p.splits = g[21]; p.p_per_split = g[22];
  TORCH_CHECK(p.Cin % chunk == 0 && p.Cout % 8 == 0, "wgrad channel alignment");
  const bool box = variant >= 0 && (variant & (1 << 26));   // box-staged (1,3,3) kernel: per-split slabs
  const bool halo = !box && variant >= 0 && (variant & 32);  // p_per_split = boxes per workgroup
  TORCH_CHECK(halo || box || p.p_per_split % 32 == 0, "p_per_split must be a multiple of 32");
  TORCH_CHECK(variant < 0 || !(variant & 4) || p.p_per_split % 64 == 0, "64-position stages need p_per_split % 64 == 0");
  p.slab = (int)slab;
  p.variant = (int)variant;
  p.dy_affine = (int)dy_affine;
  p.colsum = f32o(colsum);
  TORCH_CHECK(!dy_affine || (affine && p.ldd >= p.Cout && chunk == 8 && p.kt * p.kh * p.kw == 1),
              "Gram mode: 1x1 conv input with an affine, dy = x");
  TORCH_CHECK(!colsum.has_value() || colsum->numel() >= (int64_t)p.splits * p.Cout, "colsum slab too small");
  if (variant >= 0 && (variant & 16)) {
    TORCH_CHECK(KSEL(h, wgrad_narrow_legal)(p.Cout, p.Cin, p.K) && chunk == 8 && !slab, "narrow wgrad not legal here");
    TORCH_CHECK(p.p_per_split % 64 == 0 && (int64_t)p.splits * p.p_per_split >= p.P, "narrow wgrad: split cover");
    TORCH_CHECK(p.ldd % 8 == 0 && p.ldx % 8 == 0, "narrow wgrad: 16-B rows");
    TORCH_CHECK(!dy_affine || (p.Cout == p.Cin && p.K == p.Cin), "narrow Gram: square 1x1");
  }
  TORCH_CHECK(!halo || (KSEL(h, wgrad_halo_legal)(p) && chunk == 8 && p.p_per_split > 0), "halo wgrad not legal here");
  if (!box && variant >= 0 && (variant & (1 << 25)))
    TORCH_CHECK(KSEL(h, wgrad_rt_legal)(p.Cout, p.Cin, p.ldd, p.ldx, (int)chunk, (int)dy_affine) && p.p_per_split > 0 &&
                    (int64_t)p.splits * p.p_per_split >= p.P,
                "row-table wgrad not legal here");
  if (box) {
    TORCH_CHECK(KSEL(h, wgrad_box_legal)(p) && chunk == 8 && slab, "box wgrad not legal here (needs slab mode)");
    const int64_t boxes = p.P / (p.Wo * (int64_t)KSEL(h, wgrad_box_legal)(p));
    TORCH_CHECK(p.p_per_split > 0 && (int64_t)p.splits * p.p_per_split >= boxes, "box wgrad: split cover");
  }
  TORCH_CHECK(dy.numel() * 2 < 0xFFFFFF00ll && x.numel() * 2 < 0xFFFFFF00ll, "buffer extents must fit 32 bits");
  p.dybytes = (unsigned)(dy.numel() * 2);
  p.xbytes = (unsigned)(x.numel() * 2);
  const int64_t nslab = slab ? (int64_t)p.splits * (box && p.Cin < 64 ? 4 : 1) : 1;   // narrow box: a slab per wave
  TORCH_CHECK(partial.numel() >= (int64_t)p.Cout * p.K * nslab, "wgrad accumulator too small");
  KSEL(h, conv_wgrad_launch)(p, (int)chunk, cur_stream());
}

// slab [splits][Cout][taps*Cin] of the box kernel -> grad; tmp: >= box_reduce_groups(splits) * Cout*taps*Cin floats
void wgrad_box_reduce(const at::Tensor& slab, const at::Tensor& tmp, const at::Tensor& grad, int64_t splits,
                      int64_t Cout, int64_t taps, int64_t Cin, int64_t Cin_real, double scale, double beta) {
  const int64_t n = Cout * taps * Cin;
  TORCH_CHECK(slab.numel() >= splits * n && tmp.numel() >= pva_bf16::wgrad_box_reduce_groups((int)splits) * n && n % 4 == 0,
              "box wgrad reduce: buffer sizes");
  TORCH_CHECK(grad.numel() >= Cout * taps * Cin_real, "box wgrad reduce: grad too small");
  pva_bf16::wgrad_box_reduce_launch(f32(slab), f32(tmp), f32(grad), (int)splits, (int)Cout, (int)taps, (int)Cin, (int)Cin_real,
                          (float)scale, (float)beta, cur_stream());
}

void wgrad_reduce(const at::Tensor& partial, const at::Tensor& grad, int64_t splits, int64_t Cout, int64_t taps,
                  int64_t Cin, int64_t Cin_real, double scale, double beta, int64_t slab) {
  TORCH_CHECK(!slab || partial.numel() >= splits * Cout * taps * Cin, "slab accumulator too small");
  pva_bf16::wgrad_reduce_launch(f32(partial), f32(grad), (int)splits, (int)Cout, (int)taps, (int)Cin, (int)Cin_real,
                      (float)scale, (float)beta, (int)slab, cur_stream());
}

// Two-level finalize workspace (bn_eltwise.hip): one float64 tensor = [256][2][C] partial doubles at the front and
// ceil(C/64) zero-initialised uint32 counters (kept zero by the kernels) in its LAST doubles, so one workspace sized
// for the widest layer serves every narrower one (the executor keeps one per stream lane).  Absent: the
// single-level kernels.
inline int64_t fin_doubles(int64_t C) { return 256 * 2 * C + (C + 63) / 64; }
static void fin_buffers(const OptT& fin, int64_t C, double** scr, unsigned** ctr) {
  if (!fin.has_value()) return;
  TORCH_CHECK(fin->scalar_type() == at::kDouble && fin->is_cuda() && fin->numel() >= fin_doubles(C),
              "finalize workspace: float64 [256*2*C + C/64] on the GPU");
  *scr = fin->data_ptr<double>();
  *ctr = reinterpret_cast<unsigned*>(*scr + fin->numel() - (C + 63) / 64);
}

void bn_finalize(const at::Tensor& part, int64_t tiles, int64_t C, int64_t count, const at::Tensor& gamma,
                 const at::Tensor& beta, const OptT& rm, const OptT& rv, const OptT& nbt, double momentum, double eps,
                 const at::Tensor& smean, const at::Tensor& srstd, const at::Tensor& scale, const at::Tensor& shift,
                 const OptT& fin) {
  int64_t* nb = nbt.has_value() ? nbt->data_ptr<int64_t>() : nullptr;
  double* scr = nullptr;
  unsigned* ctr = nullptr;
  fin_buffers(fin, C, &scr, &ctr);
  pva_bf16::bn_finalize_launch(f32(part), (int)tiles, (int)C, count, f32(gamma), f32(beta), f32o(rm), f32o(rv), nb,
                     (float)momentum, (float)eps, f32(smean), f32(srstd), f32(scale), f32(shift), cur_stream(), scr, ctr);
}

void bn_eval_affine(const at::Tensor& gamma, const at::Tensor& beta, const at::Tensor& rm, const at::Tensor& rv,
                    double eps, const at::Tensor& scale, const at::Tensor& shift) {
  pva_bf16::bn_eval_affine_launch((int)gamma.numel(), f32(gamma), f32(beta), f32(rm), f32(rv), (float)eps, f32(scale),
                        f32(shift), cur_stream());
}

void bn_act(const at::Tensor& y, int64_t ldy, const at::Tensor& out, int64_t ldo, const at::Tensor& scale,
            const at::Tensor& shift, int64_t relu, int64_t M, int64_t C) {
  const bool h = kind16(y);
  TORCH_CHECK(C % 8 == 0 && ldy % 8 == 0 && ldo % 8 == 0, "bn_act alignment");
  KSEL(h, bn_act_launch)(bfp(y), (int)ldy, bfpm(out), (int)ldo, f32(scale), f32(shift), (int)relu, M, (int)C, cur_stream());
}

void res_out(const at::Tensor& yc, const at::Tensor& sc, const at::Tensor& hc, const OptT& y1, const OptT& s1,
             const OptT& h1, const OptT& x, int64_t ldx, const at::Tensor& out, int64_t ldo, int64_t M, int64_t C,
             const OptT& mask) {
  const bool h = kind16(yc);
  TORCH_CHECK(y1.has_value() || x.has_value(), "res_out needs a shortcut");
  TORCH_CHECK(!mask.has_value() || (mask->scalar_type() == at::kByte && mask->numel() >= M * (C / 8)),
              "res_out mask must be uint8 [M, C/8]");
  KSEL(h, res_out_launch)(bfp(yc), f32(sc), f32(hc), bfo(y1), f32o(s1), f32o(h1), bfo(x), (int)ldx, bfpm(out), (int)ldo,
                 mask.has_value() ? mask->data_ptr<uint8_t>() : nullptr, M, (int)C, cur_stream());
}

// mask operand of the BN-backward kernels: bf16 block output (mode 1) or uint8 ReLU bits (mode 3)
static const void* mask_ptr(int64_t mode, const OptT& mo) {
  if (mode == 1) return bfo(mo);
  if (mode == 3) {
    TORCH_CHECK(mo.has_value() && mo->scalar_type() == at::kByte, "mask mode 3 needs uint8 mask bits");
    return mo->data_ptr<uint8_t>();
  }
  return nullptr;
}

std::vector<int64_t> bn_bwd_blocks(int64_t M, int64_t C) {
  int rpb;
  int b = pva_bf16::bn_bwd_reduce_blocks(M, (int)C, &rpb);
  return {b, rpb};
}

// y0 (+mean0/rstd0) optional: without it only sum(dz) (and the y1 terms) are reduced
void bn_bwd_reduce(const at::Tensor& g, int64_t ldg, int64_t mask_mode, const OptT& mo, int64_t ldm, const OptT& ms,
                   const OptT& mh, const OptT& y0, const OptT& mean0, const OptT& rstd0,
                   const OptT& y1, const OptT& mean1, const OptT& rstd1, int64_t M, int64_t C, int64_t blocks,
                   int64_t rpb, const at::Tensor& part, const OptT& dzout, int64_t lddz) {
  const bool h = kind16(g);
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn_bwd_reduce channel constraint");
  TORCH_CHECK(!dzout.has_value() || (lddz % 8 == 0 && dzout->size(0) >= M), "bn_bwd_reduce: dz output layout");
  TORCH_CHECK(!y0.has_value() || (mean0.has_value() && rstd0.has_value()), "y0 needs mean0/rstd0");
  TORCH_CHECK(mask_mode != 2 || y0.has_value(), "mask mode 2 reads y0");
  KSEL(h, bn_bwd_reduce_launch)(bfp(g), (int)ldg, (int)mask_mode, mask_ptr(mask_mode, mo), (int)ldm, f32o(ms), f32o(mh), bfo(y0), f32o(mean0),
                       f32o(rstd0), bfo(y1), f32o(mean1), f32o(rstd1), M, (int)C, (int)blocks, (int)rpb, f32(part),
                       bfom(dzout), (int)lddz, cur_stream());
}

void bn_bwd_finalize(const at::Tensor& part, int64_t blocks, int64_t C, int64_t count, int64_t which,
                     const at::Tensor& gamma, const at::Tensor& mean, const at::Tensor& rstd, const OptT& dgamma,
                     const OptT& dbeta, double beta_acc, const at::Tensor& coef, const OptT& fin) {
  double* scr = nullptr;
  unsigned* ctr = nullptr;
  fin_buffers(fin, C, &scr, &ctr);
  pva_bf16::bn_bwd_finalize_launch(f32(part), (int)blocks, (int)C, count, (int)which, f32(gamma), f32(mean), f32(rstd),
                         f32o(dgamma), f32o(dbeta), (float)beta_acc, f32(coef), cur_stream(), scr, ctr);
}

// y0/coef0/dy0 optional (all or none): without them only dy1 and/or dz (dzout) are produced
void bn_bwd_apply(const at::Tensor& g, int64_t ldg, int64_t mask_mode, const OptT& mo, int64_t ldm, const OptT& ms,
                  const OptT& mh, const OptT& y0, const OptT& coef0, const OptT& dy0,
                  const OptT& y1, const OptT& coef1, const OptT& dy1, const OptT& dzout, int64_t lddz,
                  int64_t dz_accum, int64_t M, int64_t C) {
  const bool h = kind16(g);
  TORCH_CHECK(y0.has_value() == coef0.has_value() && y0.has_value() == dy0.has_value(), "y0/coef0/dy0 go together");
  TORCH_CHECK(mask_mode != 2 || y0.has_value(), "mask mode 2 reads y0");
  KSEL(h, bn_bwd_apply_launch)(bfp(g), (int)ldg, (int)mask_mode, mask_ptr(mask_mode, mo), (int)ldm, f32o(ms), f32o(mh), bfo(y0), f32o(coef0),
                      bfom(dy0), bfo(y1), f32o(coef1), bfom(dy1), bfom(dzout), (int)lddz, (int)dz_accum, M, (int)C,
                      cur_stream());
}

// ymax (optional, dense [NT*Ho*Wo, C] bf16): the raw y at each window's argmax, for the pooled-grid BN-backward sums
void stem_pool_fwd(const at::Tensor& y, const at::Tensor& scale, const at::Tensor& shift, const at::Tensor& out,
                   int64_t ldo, const at::Tensor& arg, int64_t NT_, int64_t H, int64_t W, int64_t Ho, int64_t Wo,
                   int64_t C, const OptT& ymax) {
  const bool h = kind16(y);
  TORCH_CHECK(C % 8 == 0 && ldo % 8 == 0, "stem pool: channels / row stride must be multiples of 8");
  TORCH_CHECK(arg.numel() >= NT_ * Ho * Wo * C, "stem pool: argmax buffer too small");
  TORCH_CHECK(!ymax.has_value() || ymax->numel() >= NT_ * Ho * Wo * C, "stem pool: ymax buffer too small");
  TORCH_CHECK(NT_ * H * W < ((int64_t)1 << 31) && C <= 2048, "stem pool: position count exceeds int32");
  TORCH_CHECK(Ho == (H - 1) / 2 + 1 && Wo == (W - 1) / 2 + 1, "stem pool: 3x3/s2/p1 output dims");
  KSEL(h, stem_pool_fwd_launch)(bfp(y), f32(scale), f32(shift), bfpm(out), arg.data_ptr<uint8_t>(), bfom(ymax), (int)NT_,
                       (int)H, (int)W, (int)Ho, (int)Wo, (int)C, (int)ldo, cur_stream());
}

// fused max-pool backward (argmax gather) + ReLU mask + BN-backward apply: dy = A*dz*mask + B*y + C
void stem_pool_bn_apply(const at::Tensor& dout, int64_t ldd, const at::Tensor& arg, const at::Tensor& y,
                        const at::Tensor& ms, const at::Tensor& mh, const at::Tensor& coef, const at::Tensor& dy,
                        int64_t NT_, int64_t H, int64_t W, int64_t Ho, int64_t Wo, int64_t C) {
  const bool h = kind16(dout);
  TORCH_CHECK(C % 8 == 0 && ldd % 8 == 0 && C <= 2048, "stem pool bwd: channel layout");
  TORCH_CHECK(NT_ * H * W < ((int64_t)1 << 31), "stem pool bwd: position count exceeds int32");
  TORCH_CHECK(y.numel() >= NT_ * H * W * C && dy.numel() >= NT_ * H * W * C, "stem pool bwd: y/dy too small");
  TORCH_CHECK(arg.numel() >= NT_ * Ho * Wo * C && dout.dim() == 2 && dout.size(0) >= NT_ * Ho * Wo &&
              dout.size(1) >= C && dout.stride(0) == ldd, "stem pool bwd: pooled buffers / row stride");
  TORCH_CHECK(Ho == (H - 1) / 2 + 1 && Wo == (W - 1) / 2 + 1, "stem pool bwd: 3x3/s2/p1 output dims");
  KSEL(h, stem_pool_bn_apply_launch)(bfp(dout), (int)ldd, arg.data_ptr<uint8_t>(), bfp(y), f32(ms), f32(mh), f32(coef), bfpm(dy),
                            (int)NT_, (int)H, (int)W, (int)Ho, (int)Wo, (int)C, cur_stream());
}

void stem_pool_bwd(const at::Tensor& dout, int64_t ldd, const at::Tensor& arg, const at::Tensor& dact, int64_t NT_,
                   int64_t H, int64_t W, int64_t Ho, int64_t Wo, int64_t C) {
  const bool h = kind16(dout);
  KSEL(h, stem_pool_bwd_launch)(bfp(dout), (int)ldd, arg.data_ptr<uint8_t>(), bfpm(dact), (int)NT_, (int)H, (int)W, (int)Ho,
                       (int)Wo, (int)C, cur_stream());
}

void avgpool_fwd(const at::Tensor& x, std::vector<int64_t> dims, std::vector<int64_t> k, const at::Tensor& out,
                 int64_t ldo, int64_t coff) {
  const bool h = kind16(x);
  const int N = (int)dims[0], T = (int)dims[1], H = (int)dims[2], W = (int)dims[3], C = (int)dims[4];
  at::Tensor scratch;
  if (k[0] == T && k[1] == H && k[2] == W)   // global pool: per-split partial sums (deterministic)
    scratch = at::empty({(int64_t)N * KSEL(h, avgpool_global_splits)(N, T * H * W) * C}, out.options());
  KSEL(h, avgpool_fwd_launch)(bfp(x), N, T, H, W, C, (int)k[0], (int)k[1], (int)k[2], f32(out), (int)ldo, (int)coff,
                     scratch.defined() ? scratch.data_ptr<float>() : nullptr, cur_stream());
}

void avgpool_bwd(const at::Tensor& dout, int64_t ldo, int64_t coff, std::vector<int64_t> dims, std::vector<int64_t> k,
                 const at::Tensor& dx) {
  const bool h = kind16(dx);
  KSEL(h, avgpool_bwd_launch)(f32(dout), (int)ldo, (int)coff, (int)dims[0], (int)dims[1], (int)dims[2], (int)dims[3],
                     (int)dims[4], (int)k[0], (int)k[1], (int)k[2], bfpm(dx), cur_stream());
}

// found_inf: raised on non-finite gradients; skip_if: when given, the step is a no-op if *skip_if != 0
// (fp16 GradScaler: nonfinite_check fills the flag first, then the update reads it on the device)
void sgd_momentum(const at::Tensor& p, const at::Tensor& g, const at::Tensor& buf, const at::Tensor& lr,
                  double momentum, double wd, double gscale, int64_t first, const OptT& found_inf,
                  const OptT& skip_if) {
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == buf.numel(), "sgd buffers must match");
  int* fi = found_inf.has_value() ? found_inf->data_ptr<int>() : nullptr;
  const int* sk = skip_if.has_value() ? skip_if->data_ptr<int>() : nullptr;
  pva_bf16::sgd_momentum_launch(f32(p), f32(g), f32(buf), p.numel(), f32(lr), (float)momentum, (float)wd, (float)gscale,
                      (int)first, fi, sk, cur_stream());
}

void nonfinite_check(const at::Tensor& g, double gscale, const at::Tensor& flag) {
  TORCH_CHECK(flag.scalar_type() == at::kInt, "flag must be int32");
  pva_bf16::nonfinite_check_launch(f32(g), g.numel(), (float)gscale, flag.data_ptr<int>(), cur_stream());
}

void pack_weights(const at::Tensor& master, const at::Tensor& fwd, const at::Tensor& dgr, const at::Tensor& descs,
                  int64_t ntensors) {
  const bool h = kind16(fwd);
  KSEL(h, pack_weights_launch)(f32(master), bfpm(fwd), bfpm(dgr), descs.data_ptr(), (int)ntensors, cur_stream());
}

// frames: packed uint8 ; desc [B,10] int32 ; tidx [B,T] int32 ; out [B*T*S*S, 4] bf16
// slow_of [T] int32 (slow frame of each frame, -1 if none) + slow_out: the slow pathway's frames, written in the same
// pass (pack_pathway_indices selects a subset of the clip's frames)
void video_preprocess(const at::Tensor& frames, const at::Tensor& desc, const at::Tensor& tidx, int64_t T, int64_t S,
                      std::vector<double> mean, std::vector<double> std_, const at::Tensor& out, bool s2d,
                      const OptT& slow_of, const OptT& slow_out, int64_t Ts) {
  const bool h = kind16(out);
  TORCH_CHECK(!s2d || S % 2 == 0, "space-to-depth output needs an even crop");
  TORCH_CHECK(frames.scalar_type() == at::kByte, "frames must be uint8");
  TORCH_CHECK(desc.dim() == 2 && desc.size(1) == 10 && desc.scalar_type() == at::kInt, "desc [B,10] int32");
  TORCH_CHECK(tidx.dim() == 2 && tidx.size(1) == T && tidx.scalar_type() == at::kInt, "tidx [B,T] int32");
  TORCH_CHECK(out.numel() >= desc.size(0) * T * S * S * 4, "output too small");
  const float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
  const float s[3] = {(float)std_[0], (float)std_[1], (float)std_[2]};
  TORCH_CHECK(slow_of.has_value() == slow_out.has_value(), "slow_of and slow_out go together");
  if (slow_of.has_value()) {
    TORCH_CHECK(slow_of->scalar_type() == at::kInt && slow_of->numel() == T, "slow_of [T] int32");
    TORCH_CHECK(slow_out->numel() >= desc.size(0) * Ts * S * S * 4 && kind16(*slow_out) == h, "slow output size / type");
  }
  KSEL(h, video_preprocess_launch)(frames.data_ptr<uint8_t>(), desc.data_ptr<int>(), tidx.data_ptr<int>(), (int)desc.size(0),
                          (int)T, (int)S, m, s, bfpm(out), s2d ? 1 : 0, cur_stream(),
                          slow_of.has_value() ? slow_of->data_ptr<int>() : nullptr, bfom(slow_out), (int)Ts);
}

// space-to-depth stems: x [N*T*Hs*Ws, 16] bf16 ; wpack [Cout_pad16, kt*256] bf16
void stem_fwd(const at::Tensor& x, const at::Tensor& wpack, const at::Tensor& y, const at::Tensor& stats,
              std::vector<int64_t> dims, int64_t Cout, int64_t kt) {
  const bool h = kind16(x);
  TORCH_CHECK(KSEL(h, stem_s2d_supported)((int)Cout, (int)kt), "unsupported stem");
  TORCH_CHECK(x.size(1) == 16 && x.is_contiguous(), "stem input must be dense s2d [M,16]");
  const int N = dims[0], T = dims[1], Hs = dims[2], Ws = dims[3];
  TORCH_CHECK(stats.numel() >= (int64_t)KSEL(h, stem_tiles)(Hs, Ws, N) * 2 * Cout, "stats too small");
  KSEL(h, stem_s2d_launch)(0, bfp(x), bfp(wpack), bfpm(y), f32(stats), nullptr, nullptr, N, T, Hs, Ws, (int)Cout, (int)kt,
                  cur_stream(), nullptr);
}

void stem_wgrad(const at::Tensor& x, const at::Tensor& dy, const at::Tensor& acc, std::vector<int64_t> dims,
                int64_t Cout, int64_t kt, const OptT& slab) {
  const bool h = kind16(x);
  TORCH_CHECK(KSEL(h, stem_s2d_supported)((int)Cout, (int)kt), "unsupported stem");
  TORCH_CHECK(acc.numel() >= Cout * kt * 256, "accumulator too small");
  const int N = dims[0], T = dims[1], Hs = dims[2], Ws = dims[3];
  // slab (reproducible mode): one partial dW per workgroup, summed in a fixed order into acc
  TORCH_CHECK(!slab.has_value() || slab->numel() >= (int64_t)KSEL(h, stem_tiles)(Hs, Ws, N) * Cout * kt * 256,
              "stem slab too small");
  KSEL(h, stem_s2d_launch)(1, bfp(x), nullptr, nullptr, nullptr, bfp(dy), f32(acc), N, T, Hs, Ws, (int)Cout, (int)kt,
                  cur_stream(), f32o(slab));
}

// ---- classification head (csrc/kernels/head.hip) ----
// feat [N][P][C] fp32, W [K][C] fp32, b [K] (nullable); xm [N][C], logits [N][K] outputs
inline const uint64_t* seed_ptr(const OptT& t) {
  if (!t.has_value()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kLong && t->numel() >= 1 && t->is_cuda(), "device seed must be int64 [1]");
  return reinterpret_cast<const uint64_t*>(t->data_ptr<int64_t>());
}

// seed_dev (optional int64 [1] on the device): the dropout key is read there instead of ``seed``
void head_forward(const at::Tensor& feat, const at::Tensor& W, const OptT& b, double p_drop, int64_t seed,
                  const at::Tensor& xm, const at::Tensor& logits, const OptT& seed_dev) {
  TORCH_CHECK(feat.dim() == 3 && feat.is_contiguous(), "feat must be [N][P][C] contiguous");
  const int N = feat.size(0), P = feat.size(1), C = feat.size(2), K = W.size(0);
  TORCH_CHECK(W.dim() == 2 && W.size(1) == C && W.is_contiguous(), "W must be [K][C]");
  TORCH_CHECK(xm.numel() >= (int64_t)N * C && logits.numel() >= (int64_t)N * K, "head outputs too small");
  TORCH_CHECK(p_drop >= 0.0 && p_drop < 1.0, "dropout probability must be in [0, 1)");
  if (N == 0) return;
  pva_bf16::head_forward_launch(f32(feat), N, P, C, f32(W), f32o(b), K, (float)p_drop, (uint64_t)seed, seed_ptr(seed_dev),
                      f32(xm), f32(logits), cur_stream());
}

// cross-entropy: loss [1] (mean over rows), dlogits (nullable) = (softmax - onehot) * gscale, counts int64 [2]
// (correct, rows; accumulated when acc_counts); rows scratch fp32 [N] + int32 [N]
void head_ce(const at::Tensor& logits, const OptT& labels, double gscale, const OptT& dlogits, const OptT& loss,
             const OptT& counts, int64_t acc_counts, const at::Tensor& row_loss, const at::Tensor& row_correct) {
  const int N = logits.size(0), K = logits.size(1);
  TORCH_CHECK(!labels.has_value() || (labels->scalar_type() == at::kLong && labels->numel() == N), "labels int64 [N]");
  TORCH_CHECK(!counts.has_value() || (counts->scalar_type() == at::kLong && counts->numel() >= 2), "counts int64 [2]");
  TORCH_CHECK(row_correct.scalar_type() == at::kInt && row_correct.numel() >= N && row_loss.numel() >= N, "row scratch");
  if (N == 0) return;
  pva_bf16::head_ce_launch(f32(logits), labels.has_value() ? labels->data_ptr<int64_t>() : nullptr, N, K, (float)gscale,
                 f32o(dlogits), f32(row_loss), row_correct.data_ptr<int>(), f32o(loss),
                 counts.has_value() ? counts->data_ptr<int64_t>() : nullptr, (int)acc_counts, cur_stream());
}

void head_backward(const at::Tensor& dlogits, const at::Tensor& xm, const at::Tensor& W, int64_t P, double p_drop,
                   int64_t seed, const at::Tensor& dW, const OptT& db, double beta, const OptT& dfeat,
                   const at::Tensor& scratch, const OptT& seed_dev) {
  const int N = dlogits.size(0), K = dlogits.size(1), C = W.size(1);
  TORCH_CHECK(xm.numel() >= (int64_t)N * C && dW.numel() == (int64_t)K * C, "head backward shapes");
  TORCH_CHECK(!dfeat.has_value() || dfeat->numel() >= (int64_t)N * P * C, "dfeat too small");
  TORCH_CHECK(scratch.numel() >= (int64_t)K * N + (int64_t)C * N + (int64_t)C * K, "head scratch too small");
  if (N == 0) return;
  float* sc = f32(scratch);
  pva_bf16::head_backward_launch(f32(dlogits), f32(xm), f32(W), N, (int)P, C, K, (float)p_drop, (uint64_t)seed,
                       seed_ptr(seed_dev), f32(dW),
                       f32o(db), (float)beta, f32o(dfeat), sc, sc + (int64_t)K * N, sc + (int64_t)K * N + (int64_t)C * N,
                       cur_stream());
}

// ---- BatchNorm folding of conv_c (csrc/kernels/bn_fold.hip) ----
void bnfold_fwd_stats(const at::Tensor& Wf, const at::Tensor& Ga, const at::Tensor& sslab, int64_t splits, int64_t C,
                      int64_t c, int64_t count, const at::Tensor& T, const at::Tensor& s_out, const at::Tensor& gamma,
                      const at::Tensor& beta, const OptT& rm, const OptT& rv, const OptT& nbt, double momentum,
                      double eps, const at::Tensor& smean, const at::Tensor& srstd, const at::Tensor& scale,
                      const at::Tensor& shift) {
  const bool h = kind16(Wf);
  TORCH_CHECK(c % 8 == 0 && c <= 2048 && Wf.numel() >= C * c && Ga.numel() >= c * c && T.numel() >= C * c,
              "bnfold_fwd_stats shapes");
  TORCH_CHECK(sslab.numel() >= splits * c && s_out.numel() >= c, "bnfold colsum shapes");
  int64_t* nb = nbt.has_value() ? nbt->data_ptr<int64_t>() : nullptr;
  KSEL(h, bnfold_fwd_stats_launch)(bfp(Wf), f32(Ga), f32(sslab), (int)splits, (int)C, (int)c, count, f32(T), f32(s_out),
                          f32(gamma), f32(beta), f32o(rm), f32o(rv), nb, (float)momentum, (float)eps, f32(smean),
                          f32(srstd), f32(scale), f32(shift), cur_stream());
}

void bnfold_bwd(const at::Tensor& part, int64_t tiles, const at::Tensor& Wf, const at::Tensor& Wd, const at::Tensor& G,
                const at::Tensor& T, const at::Tensor& s, int64_t C, int64_t c, int64_t count, const at::Tensor& gamma,
                const at::Tensor& mean, const at::Tensor& rstd, const OptT& dgamma, const OptT& dbeta,
                const at::Tensor& dW, double beta_acc, const at::Tensor& coef, const at::Tensor& W1t,
                const at::Tensor& W2, const at::Tensor& bias) {
  const bool h = kind16(Wf);
  TORCH_CHECK(c % 8 == 0 && Wf.numel() >= C * c && Wd.numel() >= C * c && G.numel() >= C * c && T.numel() >= C * c &&
              dW.numel() == C * c && coef.numel() >= 4 * C && W1t.numel() >= C * c && W2.numel() >= c * c &&
              bias.numel() >= 2 * c && part.numel() >= tiles * 3 * C, "bnfold_bwd shapes");
  KSEL(h, bnfold_bwd_launch)(f32(part), (int)tiles, bfp(Wf), bfp(Wd), f32(G), f32(T), f32(s), (int)C, (int)c, count,
                    f32(gamma), f32(mean), f32(rstd), f32o(dgamma), f32o(dbeta), f32(dW), (float)beta_acc, f32(coef),
                    bfpm(W1t), bfpm(W2), f32(bias), cur_stream());
}

void head_seed_advance(const at::Tensor& seed_dev) {
  TORCH_CHECK(seed_dev.scalar_type() == at::kLong && seed_dev.numel() >= 1 && seed_dev.is_cuda(), "int64 [1] seed");
  pva_bf16::head_seed_advance_launch(reinterpret_cast<uint64_t*>(seed_dev.data_ptr<int64_t>()), cur_stream());
}

void head_dropout_mask(const at::Tensor& out, double p_drop, int64_t seed) {
  TORCH_CHECK(out.scalar_type() == at::kByte, "mask must be uint8");
  pva_bf16::head_dropout_mask_launch(out.numel(), (float)p_drop, (uint64_t)seed, out.data_ptr<uint8_t>(), cur_stream());
}

// fused BN-backward apply + weight gradient + input gradient of a narrow 1x1 conv_c (narrow_bwd.hip)
// bn = (sb, hb, mb, rb): the input is raw conv_b output under BN_b + ReLU (mask + partial sums into part); without it
// the input is an activation used as is (branch1 of the unit: no mask, no sums) and dab may be accumulated.
// form 0: yc read from memory; 1: yc recomputed from act_b (BN-folded unit); 2: the folded unit's reduce pass (BN_c /
// BN_1 backward partial sums into cpart [splits][3][CO], rebased with mc/rc, m1/r1; nothing else written)
void narrow_c_bwd(const at::Tensor& g, int64_t ldg, int64_t mode, const OptT& mask, const OptT& yc,
                  const at::Tensor& coef, const OptT& dz, int64_t lddz, int64_t dz_accum, const at::Tensor& yb,
                  const OptT& sb, const OptT& hb, const OptT& mb, const OptT& rb, const at::Tensor& wc,
                  const OptT& dab, int64_t ldo, int64_t accum, const OptT& slab, const OptT& part, int64_t M,
                  int64_t CO, int64_t CI, int64_t rps, int64_t form, const OptT& y1, const OptT& mc, const OptT& rc,
                  const OptT& m1, const OptT& r1, const OptT& cpart) {
  const bool h = kind16(g);
  TORCH_CHECK(pva_bf16::narrow_c_bwd_legal((int)CO, (int)CI), "narrow_c_bwd: unsupported channels");
  TORCH_CHECK(mode == 0 || (mode == 3 && mask.has_value()), "narrow_c_bwd: mask mode 0 or 3 (bits)");
  TORCH_CHECK(form >= 0 && form <= 2, "narrow_c_bwd: form 0, 1 or 2");
  TORCH_CHECK(form != 0 || (yc.has_value() && yc->numel() >= M * CO), "narrow_c_bwd: form 0 reads yc");
  TORCH_CHECK(yb.numel() >= M * CI && wc.numel() >= CO * CI, "narrow_c_bwd: tensor sizes");
  TORCH_CHECK(ldg % 8 == 0 && (!dz.has_value() || lddz % 8 == 0) && ldo % 2 == 0, "narrow_c_bwd: aligned rows");
  const bool bn = sb.has_value();
  TORCH_CHECK(bn == (hb.has_value() && mb.has_value() && rb.has_value()), "narrow_c_bwd: BN_b scale/shift/mean/rstd");
  const int64_t splits = (M + rps - 1) / rps;
  if (form == 2) {
    TORCH_CHECK(bn && mc.has_value() && rc.has_value() && cpart.has_value() && cpart->numel() >= splits * 3 * CO,
                "narrow_c_bwd reduce: BN_b affine, BN_c mean/rstd and the partial-sum buffer");
    TORCH_CHECK(!y1.has_value() || (m1.has_value() && r1.has_value() && y1->numel() >= M * CO),
                "narrow_c_bwd reduce: branch1 needs its mean / rstd");
  } else {
    TORCH_CHECK(dab.has_value() && dab->numel() >= (M - 1) * ldo + CI && slab.has_value() &&
                slab->numel() >= splits * CO * CI, "narrow_c_bwd: dab / slab sizes");
    TORCH_CHECK(!bn || (part.has_value() && part->numel() >= splits * 3 * CI), "narrow_c_bwd: BN_b partial sums");
    TORCH_CHECK(!(bn && accum), "narrow_c_bwd: the BN_b-masked input gradient is written, not accumulated");
  }
  KSEL(h, narrow_c_bwd_launch)(bfp(g), (int)ldg, (int)mode, mask.has_value() ? mask->data_ptr<uint8_t>() : nullptr,
                               bfo(yc), f32(coef), bfom(dz), (int)lddz, (int)dz_accum, bfp(yb), f32o(sb), f32o(hb),
                               f32o(mb), f32o(rb), bfp(wc), bfom(dab), (int)ldo, (int)accum, f32o(slab), f32o(part),
                               bfo(y1), f32o(mc), f32o(rc), f32o(m1), f32o(r1), f32o(cpart), (int)form, M, (int)CO,
                               (int)CI, (int)rps, cur_stream());
}

// fused lateral-connection backward (csrc/kernels/lateral_bwd.hip): BN-backward apply (ReLU mask from the forward
// affine) + the strided temporal input gradient accumulated into dx; dy optionally stored for the weight gradient
void lateral_bwd(const at::Tensor& g, int64_t ldg, const at::Tensor& y, const at::Tensor& sc, const at::Tensor& sh,
                 const at::Tensor& coef, const at::Tensor& wd, const OptT& dy, const at::Tensor& dx, int64_t ldx,
                 int64_t N, int64_t To, int64_t Tf, int64_t HW, int64_t CO, int64_t Cf, int64_t alpha) {
  const bool h = kind16(g);
  TORCH_CHECK(pva_bf16::lateral_bwd_legal((int)CO, (int)Cf, (int)alpha, (int)To, (int)Tf, 7, 3),
              "lateral_bwd: unsupported geometry");
  TORCH_CHECK(ldg % 8 == 0 && ldx % 8 == 0 && ldg >= CO && ldx >= Cf, "lateral_bwd: 16-B aligned rows");
  TORCH_CHECK(y.numel() >= N * To * HW * CO && g.dim() == 2 && g.size(0) >= N * To * HW && g.size(1) >= CO &&
              g.stride(0) == ldg, "lateral_bwd: slow sizes");
  TORCH_CHECK(dx.dim() == 2 && dx.size(0) >= N * Tf * HW && dx.size(1) >= Cf && dx.stride(0) == ldx &&
              wd.numel() >= Cf * 7 * CO, "lateral_bwd: fast sizes");
  TORCH_CHECK(!dy.has_value() || dy->numel() >= N * To * HW * CO, "lateral_bwd: dy size");
  TORCH_CHECK(To * HW * ldg < (1LL << 30) && Tf * HW * ldx < (1LL << 30), "lateral_bwd: per-clip 32-bit offsets");
  KSEL(h, lateral_bwd_launch)(bfp(g), (int)ldg, bfp(y), f32(sc), f32(sh), f32(coef), bfp(wd), bfom(dy), bfpm(dx),
                              (int)ldx, (int)N, (int)To, (int)Tf, (int)HW, (int)CO, (int)Cf, (int)alpha, cur_stream());
}

void synth_frames(const at::Tensor& out, int64_t seed) {
  pva_bf16::synth_frames_launch(out.data_ptr<uint8_t>(), out.numel(), (uint32_t)seed, cur_stream());
}

}  // namespace

// generated per build by _build.py (build/obj/build_id.<id>.cpp): "PVA_BUILD_ID:" + the source-tree hash
extern "C" const char pva_build_id_str[];

PYBIND11_MODULE(_C, m) {
  m.doc() = "gfx950 HIP kernels for pytorchvideo_accelerate_amd";
  // provenance: hash of (csrc sources, headers, compile flags) this binary was linked from (_build.tree_id)
  m.def("build_id", []() { return std::string(pva_build_id_str + 13); });
  // ROCTx ranges / marks (host timeline; recorded by rocprofv3 --marker-trace, no-ops without a tool attached)
  m.def("range_push", [](const std::string& s) { return (int64_t)roctxRangePushA(s.c_str()); });
  m.def("range_pop", []() { return (int64_t)roctxRangePop(); });
  m.def("trace_mark", [](const std::string& s) { roctxMarkA(s.c_str()); });
  m.def("conv_igemm", &conv_igemm, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("stats"), py::arg("scale"),
        py::arg("shift"), py::arg("affine"), py::arg("accum"), py::arg("g"), py::arg("chunk"), py::arg("cfg") = -1,
        py::arg("bias") = py::none(), py::arg("nostore") = 0);
  m.def("conv_igemm_fres", &conv_igemm_fres);
  m.def("bnfold_fwd_stats", &bnfold_fwd_stats);
  m.def("bnfold_bwd", &bnfold_bwd);
  // launch-config helpers for the autotuner
  m.def("conv_cfg_bm", [](int64_t cfg, int64_t N) { return (int64_t)pva_bf16::conv_cfg_bm((int)cfg, (int)N); });
  m.def("conv_ut_legal", [](std::vector<int64_t> g, int64_t chunk, int64_t bk) {
    ConvParams q{};
    int* f = &q.M;
    for (int i = 0; i < 39 && i < (int)g.size(); ++i) f[i] = (int)g[i];
    return (int64_t)pva_bf16::conv_igemm_ut_legal(q, (int)chunk, (int)bk);
  });
  m.def("wgrad_halo_legal", [](std::vector<int64_t> g, int64_t variant, int64_t affine) {
    TORCH_CHECK(g.size() == 23, "wgrad geometry must have 23 entries");
    WgradParams p{};
    p.P = g[0]; p.Cout = g[1]; p.K = g[2]; p.Cin = g[3]; p.ldd = g[4]; p.ldx = g[5];
    p.Ti = g[6]; p.Hi = g[7]; p.Wi = g[8]; p.To = g[9]; p.Ho = g[10]; p.Wo = g[11];
    p.kt = g[12]; p.kh = g[13]; p.kw = g[14]; p.st = g[15]; p.sh = g[16]; p.sw = g[17];
    p.pt = g[18]; p.ph = g[19]; p.pw = g[20]; p.splits = g[21]; p.p_per_split = g[22];
    p.variant = (int)variant; p.affine = (int)affine;
    return (int64_t)pva_bf16::wgrad_halo_legal(p);
  });
  m.def("conv_pw_legal", [](std::vector<int64_t> g, int64_t chunk) {
    ConvParams q{};
    int* f = &q.M;
    for (int i = 0; i < 39 && i < (int)g.size(); ++i) f[i] = (int)g[i];
    auto dim_ok = [](int R, int as, int ao, int dir, int n, int G) {
      const int lo = ao + (dir < 0 ? -(n - 1) : 0);
      const int hi = (R - 1) * as + ao + (dir > 0 ? (n - 1) : 0);
      return n == 0 || (lo >= 0 && hi < G);
    };
    q.check = (dim_ok(q.Rt, q.ast, q.aot, q.dir, q.nt, q.Gt) && dim_ok(q.Rh, q.ash, q.aoh, q.dir, q.nh, q.Gh) &&
               dim_ok(q.Rw, q.asw, q.aow, q.dir, q.nw, q.Gw)) ? 0 : 1;
    return (int64_t)pva_bf16::conv_pw_legal(q, (int)chunk);
  });
  m.def("wgrad_box_reduce", &wgrad_box_reduce);
  m.def("box_reduce_groups", [](int64_t splits) { return (int64_t)pva_bf16::wgrad_box_reduce_groups((int)splits); });
  m.def("wgrad_box_legal", [](std::vector<int64_t> g) {
    // [P, Cout, K, Cin, ldd, ldx, Ti, Hi, Wi, To, Ho, Wo, kt, kh, kw, st, sh, sw, pt, ph, pw]
    WgradParams q{};
    q.P = g[0]; q.Cout = g[1]; q.K = g[2]; q.Cin = g[3]; q.ldd = g[4]; q.ldx = g[5];
    q.Ti = g[6]; q.Hi = g[7]; q.Wi = g[8]; q.To = g[9]; q.Ho = g[10]; q.Wo = g[11];
    q.kt = g[12]; q.kh = g[13]; q.kw = g[14]; q.st = g[15]; q.sh = g[16]; q.sw = g[17];
    q.pt = g[18]; q.ph = g[19]; q.pw = g[20];
    return (int64_t)pva_bf16::wgrad_box_legal(q);
  });
  m.def("conv_halo64p_legal", [](std::vector<int64_t> g, int64_t chunk) {
    ConvParams q{};
    int* f = &q.M;
    for (int i = 0; i < 39 && i < (int)g.size(); ++i) f[i] = (int)g[i];
    return (int64_t)pva_bf16::conv_halo64p_legal(q, (int)chunk);
  });
  m.def("conv_halo_legal", [](std::vector<int64_t> g, int64_t chunk) {
    ConvParams q{};
    int* f = &q.M;
    for (int i = 0; i < 39 && i < (int)g.size(); ++i) f[i] = (int)g[i];
    return (int64_t)pva_bf16::conv_halo_legal(q, (int)chunk);
  });
  m.def("conv_direct_legal", [](std::vector<int64_t> g, int64_t chunk) {
    ConvParams q{};
    int* f = &q.M;
    for (int i = 0; i < 39 && i < (int)g.size(); ++i) f[i] = (int)g[i];
    return (int64_t)pva_bf16::conv_direct_legal(q, (int)chunk);
  });
  m.def("conv_igemm_epi", &conv_igemm_epi, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("accum"), py::arg("g"),
        py::arg("chunk"), py::arg("res"), py::arg("ldr"), py::arg("mask"), py::arg("y0"), py::arg("mean0"),
        py::arg("rstd0"), py::arg("y1"), py::arg("mean1"), py::arg("rstd1"), py::arg("part"),
        py::arg("msc") = py::none(), py::arg("msh") = py::none(), py::arg("cfg") = -1, py::arg("bias") = py::none());
  m.def("conv_m_tiles", &conv_m_tiles, py::arg("M"), py::arg("N"), py::arg("K") = 0, py::arg("Cg") = 0);
  m.def("conv_set_bk", [](int64_t bk) { pva_bf16::conv_igemm_set_bk((int)bk); pva_f16::conv_igemm_set_bk((int)bk); });
  m.def("conv_set_ut", [](int64_t mode) { pva_bf16::conv_igemm_set_ut((int)mode); pva_f16::conv_igemm_set_ut((int)mode); });
  m.def("wgrad_rt_legal", [](int64_t Cout, int64_t Cin, int64_t ldd, int64_t ldx, int64_t chunk) {
    return pva_bf16::wgrad_rt_legal((int)Cout, (int)Cin, (int)ldd, (int)ldx, (int)chunk, 0) != 0;
  });
  m.def("wgrad_tile", &wgrad_tile, py::arg("Cout"), py::arg("K"), py::arg("variant") = -1);
  m.def("wgrad_narrow_legal", [](int64_t Cout, int64_t Cin, int64_t K) {
    return (bool)pva_bf16::wgrad_narrow_legal((int)Cout, (int)Cin, (int)K);
  });
  m.def("conv_wgrad", &conv_wgrad, py::arg("dy"), py::arg("x"), py::arg("partial"), py::arg("scale"),
        py::arg("shift"), py::arg("affine"), py::arg("g"), py::arg("chunk"), py::arg("slab") = 0,
        py::arg("variant") = -1, py::arg("dy_affine") = 0, py::arg("colsum") = py::none());
  m.def("wgrad_reduce", &wgrad_reduce, py::arg("partial"), py::arg("grad"), py::arg("splits"), py::arg("Cout"),
        py::arg("taps"), py::arg("Cin"), py::arg("Cin_real"), py::arg("scale"), py::arg("beta"), py::arg("slab") = 0);
  m.def("bn_finalize", &bn_finalize, py::arg("part"), py::arg("tiles"), py::arg("C"), py::arg("count"),
        py::arg("gamma"), py::arg("beta"), py::arg("rm"), py::arg("rv"), py::arg("nbt"), py::arg("momentum"),
        py::arg("eps"), py::arg("smean"), py::arg("srstd"), py::arg("scale"), py::arg("shift"),
        py::arg("fin") = py::none());
  m.def("fin_doubles", [](int64_t C) { return fin_doubles(C); });
  m.def("bn_eval_affine", &bn_eval_affine);
  m.def("bn_act", &bn_act);
  m.def("res_out", &res_out);
  m.def("bn_bwd_blocks", &bn_bwd_blocks);
  m.def("bn_bwd_reduce", &bn_bwd_reduce, py::arg("g"), py::arg("ldg"), py::arg("mask_mode"), py::arg("mo"),
        py::arg("ldm"), py::arg("ms"), py::arg("mh"), py::arg("y0"), py::arg("mean0"), py::arg("rstd0"), py::arg("y1"),
        py::arg("mean1"), py::arg("rstd1"), py::arg("M"), py::arg("C"), py::arg("blocks"), py::arg("rpb"),
        py::arg("part"), py::arg("dzout") = py::none(), py::arg("lddz") = 0);
  m.def("bn_bwd_finalize", &bn_bwd_finalize, py::arg("part"), py::arg("blocks"), py::arg("C"), py::arg("count"),
        py::arg("which"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"), py::arg("dgamma"), py::arg("dbeta"),
        py::arg("beta_acc"), py::arg("coef"), py::arg("fin") = py::none());
  m.def("bn_bwd_apply", &bn_bwd_apply);
  m.def("stem_pool_fwd", &stem_pool_fwd, py::arg("y"), py::arg("scale"), py::arg("shift"), py::arg("out"),
        py::arg("ldo"), py::arg("arg"), py::arg("NT"), py::arg("H"), py::arg("W"), py::arg("Ho"), py::arg("Wo"),
        py::arg("C"), py::arg("ymax") = py::none());
  m.def("stem_pool_bn_apply", &stem_pool_bn_apply);
  m.def("stem_pool_bwd", &stem_pool_bwd);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("sgd_momentum", &sgd_momentum, py::arg("p"), py::arg("g"), py::arg("buf"), py::arg("lr"),
        py::arg("momentum"), py::arg("wd"), py::arg("gscale"), py::arg("first"), py::arg("found_inf"),
        py::arg("skip_if") = py::none());
  m.def("nonfinite_check", &nonfinite_check);
  m.def("pack_weights", &pack_weights);
  m.def("pack_desc_size", &pva_bf16::pack_desc_size);
  m.def("video_preprocess", &video_preprocess, py::arg("frames"), py::arg("desc"), py::arg("tidx"), py::arg("T"),
        py::arg("S"), py::arg("mean"), py::arg("std"), py::arg("out"), py::arg("s2d"), py::arg("slow_of") = py::none(),
        py::arg("slow_out") = py::none(), py::arg("Ts") = 0);
  m.def("synth_frames", &synth_frames);
  m.def("narrow_c_bwd", &narrow_c_bwd, py::arg("g"), py::arg("ldg"), py::arg("mode"), py::arg("mask"), py::arg("yc"),
        py::arg("coef"), py::arg("dz"), py::arg("lddz"), py::arg("dz_accum"), py::arg("yb"), py::arg("sb"),
        py::arg("hb"), py::arg("mb"), py::arg("rb"), py::arg("wc"), py::arg("dab"), py::arg("ldo"), py::arg("accum"),
        py::arg("slab"), py::arg("part"), py::arg("M"), py::arg("CO"), py::arg("CI"), py::arg("rps"),
        py::arg("form") = 0, py::arg("y1") = py::none(), py::arg("mc") = py::none(), py::arg("rc") = py::none(),
        py::arg("m1") = py::none(), py::arg("r1") = py::none(), py::arg("cpart") = py::none());
  m.def("lateral_bwd", &lateral_bwd);
  m.def("lateral_bwd_legal", [](int64_t CO, int64_t Cf, int64_t alpha, int64_t To, int64_t Tf, int64_t kt, int64_t pad) {
    return (bool)pva_bf16::lateral_bwd_legal((int)CO, (int)Cf, (int)alpha, (int)To, (int)Tf, (int)kt, (int)pad);
  });
  m.def("narrow_c_bwd_legal", [](int64_t CO, int64_t CI) { return (bool)pva_bf16::narrow_c_bwd_legal((int)CO, (int)CI); });
  m.def("narrow_c_bwd_rps", [](int64_t M, int64_t CO, int64_t splits) {
    return (int64_t)pva_bf16::narrow_c_bwd_rps(M, (int)CO, (int)splits);
  });
  m.def("stem_tiles", [](int64_t Ho, int64_t Wo, int64_t N) { return pva_bf16::stem_tiles((int)Ho, (int)Wo, (int)N); });
  m.def("stem_supported", [](int64_t Cout, int64_t kt) { return pva_bf16::stem_s2d_supported((int)Cout, (int)kt); });
  m.def("head_forward", &head_forward, py::arg("feat"), py::arg("W"), py::arg("b"), py::arg("p_drop"), py::arg("seed"),
        py::arg("xm"), py::arg("logits"), py::arg("seed_dev") = py::none());
  m.def("head_seed_advance", &head_seed_advance);
  m.def("head_ce", &head_ce);
  m.def("head_backward", &head_backward, py::arg("dlogits"), py::arg("xm"), py::arg("W"), py::arg("P"),
        py::arg("p_drop"), py::arg("seed"), py::arg("dW"), py::arg("db"), py::arg("beta"), py::arg("dfeat"),
        py::arg("scratch"), py::arg("seed_dev") = py::none());
  m.def("head_dropout_mask", &head_dropout_mask);
  m.def("stem_fwd", &stem_fwd);
  m.def("stem_wgrad", &stem_wgrad, py::arg("x"), py::arg("dy"), py::arg("acc"), py::arg("dims"), py::arg("Cout"),
        py::arg("kt"), py::arg("slab") = py::none());
  m.def("stem_wgrad_convert", [](const at::Tensor& acc, const at::Tensor& grad, int64_t Cout, int64_t kt, double beta) {
    pva_bf16::stem_wgrad_convert_launch(f32(acc), f32(grad), (int)Cout, (int)kt, (float)beta, cur_stream());
  });
  m.def("stem_pack", [](const at::Tensor& w, const at::Tensor& out, int64_t Cout, int64_t kt) {
    const bool h = kind16(out);
    KSEL(h, stem_pack_launch)(f32(w), bfpm(out), (int)Cout, (int)kt, cur_stream());
  });
  register_clip_reader(m);
  register_rccl(m);
  register_fp32(m);
}
