// pybind11 bindings of the fp32 kernels (csrc/fp32/*.hip) as the submodule ``_C.f32``.
//
// Allocation-free launch shims on PyTorch's current HIP stream, like bindings.cpp.  Every launch checks what the
// kernel assumes (fp32 GPU tensors, 16-B aligned float4 rows, channel counts multiple of 4, and that the rows it
// will touch lie inside the tensors it was given) before anything reaches the GPU.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include "../fp32/launchers32.h"
#include <algorithm>
#include <cstddef>

static_assert(offsetof(Conv32, orw) - offsetof(Conv32, ldx) == 25 * sizeof(int), "Conv32 integer block contiguous");
static_assert(offsetof(Wgrad32, sw) - offsetof(Wgrad32, ldd) == 15 * sizeof(int), "Wgrad32 integer block contiguous");

namespace {

using OptT = c10::optional<at::Tensor>;

inline hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

inline float* fp(const at::Tensor& t, const char* name, bool align16 = true) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat, name, " must be an fp32 GPU tensor");
  TORCH_CHECK(!align16 || reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-B aligned");
  return t.data_ptr<float>();
}
inline float* fpo(const OptT& t, const char* name, bool align16 = true) {
  return t.has_value() ? fp(*t, name, align16) : nullptr;
}
// elements reachable from t.data_ptr() (t may be a channel-slice view of a larger buffer)
inline int64_t span(const at::Tensor& t) {
  return t.storage().nbytes() / 4 - t.storage_offset();
}

void conv32(const at::Tensor& x, const at::Tensor& w, const at::Tensor& y, const at::Tensor& taps,
            std::vector<int64_t> g, const OptT& isc, const OptT& ish, int64_t irelu, int64_t np, const OptT& stats) {
  TORCH_CHECK(np == 2 || np == 3, "conv32: np (bf16 pieces per fp32 operand) must be 2 or 3");
  TORCH_CHECK(g.size() == 26, "conv32 geometry has 26 entries");
  Conv32 p{};
  p.x = fp(x, "x");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.numel() % 3 == 0,
              "conv32: w must be the three bf16 weight planes of wpack32 (mode 0 / 1)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0, "w must be 16-B aligned");
  p.w = reinterpret_cast<const uint16_t*>(w.data_ptr());
  TORCH_CHECK(w.numel() / 3 * 6 < (int64_t(1) << 31), "conv32: weight planes exceed 2 GB");
  p.wplane = (int)(w.numel() / 3);
  p.y = fp(y, "y");
  TORCH_CHECK(taps.is_cuda() && taps.scalar_type() == at::kInt, "taps must be int32 GPU");
  p.taps = taps.data_ptr<int>();
  p.isc = fpo(isc, "isc");
  p.ish = fpo(ish, "ish");
  TORCH_CHECK((p.isc == nullptr) == (p.ish == nullptr), "input affine needs scale and shift");
  p.irelu = (int)irelu;
  int* f = &p.ldx;
  for (int i = 0; i < 26; ++i) f[i] = (int)g[i];
  TORCH_CHECK(p.ldx % 4 == 0 && p.ldy % 4 == 0 && p.ldw % 4 == 0 && p.Cr % 4 == 0 && p.N % 4 == 0 && p.K % 4 == 0,
              "conv32: ld / channel counts must be multiples of 4");
  TORCH_CHECK(p.Cr > 0 && p.K % p.Cr == 0 && taps.numel() >= 4 * (p.K / p.Cr), "conv32: taps table too short");
  const int64_t Q = (int64_t)p.Qt * p.Qh * p.Qw;
  TORCH_CHECK(Q > 0 && p.M % Q == 0, "conv32: M must be a whole number of position grids");
  const int64_t nb = p.M / Q;
  TORCH_CHECK(span(x) >= (nb * p.Ti * p.Hi * p.Wi - 1) * p.ldx + p.Cr || p.M == 0, "conv32: x too small");
  TORCH_CHECK(span(y) >= (nb * p.Yt * p.Yh * p.Yw - 1) * p.ldy + p.N || p.M == 0, "conv32: y too small");
  TORCH_CHECK((int64_t)p.wplane >= ((int64_t)p.N - 1) * p.ldw + p.K || p.N == 0, "conv32: w too small");
  {  // the A loads address the clips one tile's rows read through a buffer resource with a 32-bit byte range
    const int64_t bm = pva_f32::igemm32_bm(p.N), clips = std::min<int64_t>(nb, bm / Q + 2);
    TORCH_CHECK(clips * p.Ti * p.Hi * p.Wi * (int64_t)p.ldx * 4 < (int64_t(1) << 31),
                "conv32: one tile's input clips exceed the 2 GB buffer range");
  }
  TORCH_CHECK((p.Qt - 1) * p.ost + p.ort < p.Yt && (p.Qh - 1) * p.osh + p.orh < p.Yh &&
                  (p.Qw - 1) * p.osw + p.orw < p.Yw,
              "conv32: output grid exceeds the output tensor");
  p.stats = fpo(stats, "stats", false);
  if (p.stats != nullptr) {
    const int64_t tiles = (p.M + pva_f32::igemm32_bm(p.N) - 1) / pva_f32::igemm32_bm(p.N);
    TORCH_CHECK(stats->numel() >= tiles * 2 * p.N && !p.accum, "conv32: stats needs [M tiles][2][N], no accumulate");
  }
  pva_f32::igemm32_launch(p, (int)np, stream());
}

void wgrad32(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& dw, const at::Tensor& taps,
             std::vector<int64_t> g, const OptT& isc, const OptT& ish, int64_t irelu, int64_t np) {
  TORCH_CHECK(np == 2 || np == 3, "wgrad32: np (bf16 pieces per fp32 operand) must be 2 or 3");
  TORCH_CHECK(g.size() == 16, "wgrad32 geometry has 16 entries");
  Wgrad32 p{};
  p.dy = fp(dy, "dy");
  p.x = fp(x, "x");
  p.dw = fp(dw, "dw", false);
  TORCH_CHECK(taps.is_cuda() && taps.scalar_type() == at::kInt, "taps must be int32 GPU");
  p.taps = taps.data_ptr<int>();
  p.isc = fpo(isc, "isc");
  p.ish = fpo(ish, "ish");
  TORCH_CHECK((p.isc == nullptr) == (p.ish == nullptr), "input affine needs scale and shift");
  p.irelu = (int)irelu;
  int* f = &p.ldd;
  for (int i = 0; i < 16; ++i) f[i] = (int)g[i];
  TORCH_CHECK(p.ldd % 4 == 0 && p.ldx % 4 == 0 && p.Cout % 4 == 0 && p.Cin % 4 == 0 && p.K % p.Cin == 0,
              "wgrad32: ld / channel counts must be multiples of 4");
  TORCH_CHECK(taps.numel() >= 4 * (p.K / p.Cin), "wgrad32: taps table too short");
  const int64_t Q = (int64_t)p.Qt * p.Qh * p.Qw;
  TORCH_CHECK(Q > 0 && p.P % Q == 0, "wgrad32: P must be a whole number of position grids");
  TORCH_CHECK(span(dy) >= ((int64_t)p.P - 1) * p.ldd + p.Cout || p.P == 0, "wgrad32: dy too small");
  TORCH_CHECK(span(x) >= ((p.P / Q) * p.Ti * p.Hi * p.Wi - 1) * p.ldx + p.Cin || p.P == 0, "wgrad32: x too small");
  TORCH_CHECK(dw.numel() >= ((int64_t)p.Cout - 1) * p.ldw + p.K, "wgrad32: dw too small");
  pva_f32::wgrad32_launch(p, (int)np, stream());
}

}  // namespace

void register_fp32(pybind11::module& m) {
  namespace py = pybind11;
  auto f = m.def_submodule("f32", "fp32 (split-bf16 MFMA) kernels of the --mixed_precision no path");
  f.def("conv32", &conv32, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("taps"), py::arg("geo"),
        py::arg("isc") = py::none(), py::arg("ish") = py::none(), py::arg("irelu") = 0, py::arg("np") = 3,
        py::arg("stats") = py::none());
  f.def("igemm32_bm", [](int64_t N) { return (int64_t)pva_f32::igemm32_bm((int)N); });
  f.def("wgrad32", &wgrad32, py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("taps"), py::arg("geo"),
        py::arg("isc") = py::none(), py::arg("ish") = py::none(), py::arg("irelu") = 0, py::arg("np") = 3);
  f.def("igemm32_tile", [](int64_t N) { return (int64_t)pva_f32::igemm32_tile((int)N); });
  f.def("wgrad32_tile", [](int64_t K, int64_t Cout) {
    int a, b;
    pva_f32::wgrad32_tile((int)K, (int)Cout, &a, &b);
    return std::make_tuple((int64_t)a, (int64_t)b);
  });
  f.def("wpack32", [](int64_t mode, const at::Tensor& src, const at::Tensor& dst, int64_t Cout, int64_t Cin,
                      int64_t taps, int64_t cip, double beta) {
    const int64_t n = mode == 1 ? Cout * taps * Cin : mode == 0 ? Cout * taps * cip : Cout * Cin * taps;
    const int64_t ns = mode == 2 ? Cout * taps * cip : Cout * Cin * taps;
    void* d;
    if (mode == 2) {   // gradient unpack: fp32 torch layout
      TORCH_CHECK(dst.numel() >= n, "wpack32: sizes");
      d = fp(dst, "dst", false);
    } else {           // forward / input-gradient B rows: three bf16 planes of n elements
      TORCH_CHECK(dst.is_cuda() && dst.scalar_type() == at::kBFloat16 && dst.is_contiguous() && dst.numel() == 3 * n,
                  "wpack32: mode 0 / 1 write three bf16 planes of the packed rows");
      d = dst.data_ptr();
    }
    TORCH_CHECK(src.numel() >= ns && cip >= Cin, "wpack32: sizes");
    pva_f32::wpack32_launch((int)mode, fp(src, "src", false), d, (int)Cout, (int)Cin, (int)taps, (int)cip,
                            (float)beta, stream());
  });
  f.def("chan_reduce32_blocks", [](int64_t M, int64_t C) { return (int64_t)pva_f32::chan_reduce32_blocks(M, (int)C); });
  f.def("chan_reduce32", [](const at::Tensor& y, int64_t ldy, const OptT& d, int64_t ldd, const OptT& o, int64_t ldo,
                            const OptT& mean, int64_t mode, int64_t relu, int64_t M, int64_t C, const at::Tensor& part) {
    TORCH_CHECK(C % 4 == 0 && ldy % 4 == 0 && ldd % 4 == 0 && ldo % 4 == 0, "chan_reduce32: multiples of 4");
    TORCH_CHECK(mode == 3 ? (part.numel() >= part.size(0) * C && C % 8 == 0)
                          : (part.dim() == 3 && part.size(1) == 2 && part.size(2) == C),
                "part must be [blocks][2][C] ([blocks][C] column sums in mode 3)");
    TORCH_CHECK(span(y) >= (M - 1) * ldy + C || M == 0, "chan_reduce32: y too small");
    TORCH_CHECK(mode == 0 || mode == 3 || (d.has_value() && mean.has_value()), "chan_reduce32 args");
    // relu without o: the mask comes from the [4][C] forward statistics that mean is row 0 of
    TORCH_CHECK(mode != 1 || !relu || o.has_value() || span(*mean) >= 4 * C, "chan_reduce32: mask needs o or stat");
    pva_f32::chan_reduce32_launch(fp(y, "y"), (int)ldy, fpo(d, "d"), (int)ldd, fpo(o, "o"), (int)ldo,
                                  fpo(mean, "mean"), (int)mode, (int)relu, M, (int)C, (int)part.size(0),
                                  fp(part, "part"), stream());
  });
  f.def("bn32_finalize", [](const OptT& part, int64_t C, int64_t count, int64_t mode, const OptT& gamma,
                            const OptT& beta, const OptT& rm, const OptT& rv, const OptT& nbt, double momentum,
                            double eps, const OptT& stat, const OptT& fstat, const OptT& dgamma, const OptT& dbeta,
                            const OptT& coef, double gbeta) {
    TORCH_CHECK(mode == 2 || (part.has_value() && part->size(2) == C), "bn32_finalize: partials");
    TORCH_CHECK(mode != 1 || (fstat.has_value() && coef.has_value()), "bn32_finalize: backward needs fstat and coef");
    TORCH_CHECK(mode == 1 || (stat.has_value() && stat->numel() >= 4 * C), "bn32_finalize: stat [4][C]");
    TORCH_CHECK(mode != 2 || (rm.has_value() && rv.has_value()), "bn32_finalize: eval needs running statistics");
    int64_t* nb = nullptr;
    if (nbt.has_value()) {
      TORCH_CHECK(nbt->scalar_type() == at::kLong && nbt->is_cuda(), "nbt int64 GPU");
      nb = nbt->data_ptr<int64_t>();
    }
    pva_f32::bn32_finalize_launch(part.has_value() ? fp(*part, "part") : nullptr,
                                  part.has_value() ? (int)part->size(0) : 0, (int)C, count, (int)mode,
                                  fpo(gamma, "gamma", false), fpo(beta, "beta", false), fpo(rm, "rm", false),
                                  fpo(rv, "rv", false), nb, (float)momentum, (float)eps, fpo(stat, "stat"),
                                  fpo(fstat, "fstat"), fpo(dgamma, "dgamma", false), fpo(dbeta, "dbeta", false),
                                  fpo(coef, "coef"), (float)gbeta, stream());
  });
  f.def("bn32_apply", [](const at::Tensor& y, int64_t ldy, const at::Tensor& stat, const OptT& add, int64_t lda,
                         int64_t relu, const at::Tensor& out, int64_t ldo, int64_t M, int64_t C) {
    TORCH_CHECK(C % 4 == 0 && ldy % 4 == 0 && lda % 4 == 0 && ldo % 4 == 0 && stat.numel() >= 4 * C, "bn32_apply");
    TORCH_CHECK(span(y) >= (M - 1) * ldy + C && span(out) >= (M - 1) * ldo + C || M == 0, "bn32_apply: sizes");
    TORCH_CHECK(!add.has_value() || span(*add) >= (M - 1) * lda + C || M == 0, "bn32_apply: add too small");
    pva_f32::bn32_apply_launch(fp(y, "y"), (int)ldy, fp(stat, "stat"), fpo(add, "add"), (int)lda, (int)relu,
                               fp(out, "out"), (int)ldo, M, (int)C, stream());
  });
  f.def("bn32_bwd_apply", [](const at::Tensor& d, int64_t ldd, const OptT& o, int64_t ldo, int64_t relu,
                             const at::Tensor& y, int64_t ldy, const at::Tensor& fstat, const at::Tensor& coef,
                             const at::Tensor& dy, int64_t lddy, const OptT& gout, int64_t ldg, int64_t M, int64_t C) {
    TORCH_CHECK(C % 4 == 0 && ldd % 4 == 0 && ldo % 4 == 0 && ldy % 4 == 0 && lddy % 4 == 0 && ldg % 4 == 0,
                "bn32_bwd_apply: multiples of 4");
    TORCH_CHECK(fstat.numel() >= 4 * C, "bn32_bwd_apply: fstat [4][C]");   // (relu without o: mask from fstat)
    TORCH_CHECK(M == 0 || (span(d) >= (M - 1) * ldd + C && span(y) >= (M - 1) * ldy + C &&
                           span(dy) >= (M - 1) * lddy + C),
                "bn32_bwd_apply: sizes");
    pva_f32::bn32_bwd_apply_launch(fp(d, "d"), (int)ldd, fpo(o, "o"), (int)ldo, (int)relu, fp(y, "y"), (int)ldy,
                                   fp(fstat, "fstat"), fp(coef, "coef"), fp(dy, "dy"), (int)lddy, fpo(gout, "gout"),
                                   (int)ldg, M, (int)C, stream());
  });
  f.def("copy32", [](const at::Tensor& src, int64_t lds, const at::Tensor& dst, int64_t ldd, int64_t M, int64_t C,
                     int64_t acc) {
    TORCH_CHECK(C % 4 == 0 && lds % 4 == 0 && ldd % 4 == 0, "copy32: multiples of 4");
    TORCH_CHECK(M == 0 || (span(src) >= (M - 1) * lds + C && span(dst) >= (M - 1) * ldd + C), "copy32: sizes");
    pva_f32::copy32_launch(fp(src, "src"), (int)lds, fp(dst, "dst"), (int)ldd, M, (int)C, (int)acc, stream());
  });
  f.def("maxpool32", [](int64_t bwd, const at::Tensor& a, const at::Tensor& b, const at::Tensor& arg,
                        std::vector<int64_t> dims, std::vector<int64_t> k, std::vector<int64_t> s,
                        std::vector<int64_t> p) {
    TORCH_CHECK(dims.size() == 8 && k.size() == 3 && s.size() == 3 && p.size() == 3, "maxpool32 dims");
    const int64_t nin = dims[0] * dims[1] * dims[2] * dims[3] * dims[7];
    const int64_t nout = dims[0] * dims[4] * dims[5] * dims[6] * dims[7];
    TORCH_CHECK(k[0] * k[1] * k[2] <= 255, "maxpool32: window too large for uint8 indices");
    TORCH_CHECK(arg.scalar_type() == at::kByte && arg.numel() >= nout, "maxpool32: arg uint8 [out]");
    TORCH_CHECK(a.numel() >= (bwd ? nout : nin) && b.numel() >= (bwd ? nin : nout), "maxpool32: sizes");
    int kk[3], ss[3], pp[3];
    for (int i = 0; i < 3; ++i) { kk[i] = (int)k[i]; ss[i] = (int)s[i]; pp[i] = (int)p[i]; }
    pva_f32::maxpool32_launch((int)bwd, fp(a, "a", false), fp(b, "b", false), arg.data_ptr<uint8_t>(), (int)dims[0],
                              (int)dims[1], (int)dims[2], (int)dims[3], (int)dims[4], (int)dims[5], (int)dims[6],
                              (int)dims[7], kk, ss, pp, stream());
  });
  f.def("avgpool32", [](int64_t bwd, const at::Tensor& a, const at::Tensor& b, std::vector<int64_t> dims,
                        std::vector<int64_t> k, int64_t ldf, int64_t coff) {
    TORCH_CHECK(dims.size() == 5 && k.size() == 3, "avgpool32 dims");
    const int64_t N = dims[0], T = dims[1], H = dims[2], W = dims[3], C = dims[4];
    TORCH_CHECK(k[0] <= T && k[1] <= H && k[2] <= W && coff + C <= ldf, "avgpool32: window / channel offset");
    const int64_t P = (T - k[0] + 1) * (H - k[1] + 1) * (W - k[2] + 1);
    const int64_t nx = N * T * H * W * C, nf = N * P * ldf;
    TORCH_CHECK(a.numel() >= (bwd ? nf : nx) && b.numel() >= (bwd ? nx : nf), "avgpool32: sizes");
    pva_f32::avgpool32_launch((int)bwd, fp(a, "a", false), fp(b, "b", false), (int)N, (int)T, (int)H, (int)W, (int)C,
                              (int)k[0], (int)k[1], (int)k[2], (int)ldf, (int)coff, stream());
  });
  // zero a buffer (the weight-gradient atomics accumulate into it): a DMA memset, no fill kernel
  f.def("zero32", [](const at::Tensor& t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "zero32: contiguous GPU tensor");
    TORCH_CHECK(hipMemsetAsync(t.data_ptr(), 0, t.numel() * t.element_size(), stream()) == hipSuccess, "zero32");
  });
  f.def("to_ndhwc32", [](const at::Tensor& x, const at::Tensor& y, int64_t N, int64_t Cin, int64_t S, int64_t Cp) {
    TORCH_CHECK(x.numel() >= N * Cin * S && y.numel() >= N * S * Cp && Cp >= Cin, "to_ndhwc32: sizes");
    pva_f32::to_ndhwc32_launch(fp(x, "x", false), fp(y, "y", false), (int)N, (int)Cin, S, (int)Cp, stream());
  });
}
