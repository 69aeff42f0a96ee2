// Pointwise (1x1x1, unit-stride, unpadded) convolution: legality, launch geometry and dispatch.  The
// kernel itself (design notes at its head) is in conv_pw_impl.h, instantiated per K-step count in
// conv_pw_ks{1,2,4,8}.hip.
#include "common.h"
#include "conv_params.h"
#include <algorithm>
#include <cstdio>
#include <stdexcept>

PVA_NS_BEGIN

bool conv_pw_run_ks1(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st);
bool conv_pw_run_ks2(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st);
bool conv_pw_run_ks4(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st);
bool conv_pw_run_ks8(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st);
bool conv_pw_run_ks1_w4(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st);
bool conv_pw_run_ks2_w4(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st);
bool conv_pw_run_ks4_w4(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st);
bool conv_pw_run_ks8_w4(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st);

namespace {
constexpr int PW_LDS = 156 * 1024;     // LDS budget of a workgroup (weights, statistics, constants)
constexpr int OP_OLD = 1, OP_RES = 2, OP_Y0 = 4, OP_Y1 = 8, OP_MASK = 16, OP_MSC = 32;   // = conv_pw_impl.h

inline int pw_ks(int K) {
  const int s = (K + 31) / 32;
  return s <= 1 ? 1 : s <= 2 ? 2 : s <= 4 ? 4 : 8;
}
}  // namespace

// rows per workgroup of a pointwise launch configuration (cfg bits 0-1)
int conv_pw_rows(int cfg) { return 1024 << (cfg & 3); }

// 1 when the geometry is a dense 1x1x1 unit-stride unpadded GEMM the pointwise kernel can run, or a (kt,1,1)
// temporal conv at unit stride (forward, or the stride-1 dgrad gathering backwards) whose taps are visited in
// weight order: K = kt x Cg <= 256, clip slices of >= 32 pixels (a 64-row tile crosses at most two)
int conv_pw_legal(const ConvParams& p, int chunk) {
  if (chunk != 8) return 0;
  if (p.nh != 1 || p.nw != 1) return 0;
  if (p.ast != 1 || p.ash != 1 || p.asw != 1 || p.aoh != 0 || p.aow != 0) return 0;
  if (p.Gt != p.Rt || p.Gh != p.Rh || p.Gw != p.Rw) return 0;
  if (p.ost != 1 || p.osh != 1 || p.osw != 1 || p.ort != 0 || p.orh != 0 || p.orw != 0) return 0;
  if (p.Ot != p.Rt || p.Oh != p.Rh || p.Ow != p.Rw) return 0;
  if (p.nt == 1) {
    if (p.check || p.aot != 0) return 0;
  } else {
    if (p.bt0 != 0 || p.bts != 1 || (p.dir != 1 && p.dir != -1) || p.Rh * p.Rw < 32 || p.Rt < 2) return 0;
  }
  if (p.Kfull != p.nt * p.Cg || p.Cg % 8 != 0 || p.Kfull > 256 || p.Ngemm % 32 != 0) return 0;
  if (p.ldx % 8 != 0 || p.ldy % 8 != 0) return 0;
  return 1;
}

// 32-channel chunks per output-channel group: the largest group whose weight image, statistics and epilogue
// constants fit the LDS budget, then balanced over the groups (equal work per workgroup)
static int pw_group_chunks(int N, int ks, int nslot, int aff_bytes, int budget) {
  const int nch = N / 32;
  const int per_chunk = 2 * ks * 1024 + (nslot + 4) * 32 * 4;
  int gmax = std::max(1, (budget - aff_bytes) / per_chunk);
  if (gmax >= 2) gmax &= ~1;   // even groups: chunk pairs stay aligned to 128-B lines
  const int ngrp = (nch + gmax - 1) / gmax;
  const int g = (nch + ngrp - 1) / ngrp;
  return (nch >= 2 && gmax >= 2) ? (g + 1) & ~1 : g;
}

void conv_pw_launch(const ConvParams& p, int cfg, hipStream_t st) {
  const bool ep2 = !p.fres && (p.eres || p.emask || p.epart);
  const int ep = p.fres ? 1 : (ep2 ? 2 : 0);
  const int ks = pw_ks(p.Kfull);
  // cfg bit 3: 4-wave workgroups, their LDS budget halved so that at least two share a CU
  const bool w4 = (cfg & 8) != 0;
  const int nw = w4 ? 4 : 8;
  // per-wave statistic slots [waves][statistics] per channel (none for the residual output)
  const int nslot = ep == 1 ? 0 : (ep == 2 ? 3 : 2) * nw;
  const int aff_bytes = p.affine ? 2 * p.Cg * 4 : 0;
  const int gch = pw_group_chunks(p.Ngemm, ks, nslot, aff_bytes, w4 ? PW_LDS / 2 : PW_LDS);
  const int NG = gch * 32;
  size_t lds = (size_t)gch * 2 * ks * 1024 + (size_t)(nslot + 4) * NG * 4 + aff_bytes;
  // cfg bit 2: one workgroup per CU (the LDS request is padded past half the CU's LDS).  Instantiations
  // under 128 VGPRs otherwise run two per CU, which measured slower on some streaming shapes
  // (more rows in flight thrash the L2 / DRAM pages) and faster on others: the autotuner picks
  if (cfg & 4) lds = std::max(lds, (size_t)(84 * 1024));
  const int rpb = conv_pw_rows(cfg);
  // operand streams of the epilogue (the kernel is instantiated per combination)
  const bool stats2 = ep == 2 && p.epart != nullptr;
  int ops = p.accum && ep != 1 ? OP_OLD : 0;
  if (ep == 1 && p.rsc) ops |= 64;   // OP_RAFF: BN_1 affine on the residual
  if (ep == 2) {
    if (p.eres) ops |= OP_RES;
    if (p.emask) ops |= OP_MASK;
    if (p.emsc) ops |= OP_MSC;
    if (p.ey0 && (p.emsc || stats2)) ops |= OP_Y0;
    if (p.ey1 && stats2) ops |= OP_Y1;
  }
  bool ok;
  switch (ks * (w4 ? -1 : 1)) {
    case 1: ok = conv_pw_run_ks1(p, ep, ops, rpb, gch, lds, st); break;
    case 2: ok = conv_pw_run_ks2(p, ep, ops, rpb, gch, lds, st); break;
    case 4: ok = conv_pw_run_ks4(p, ep, ops, rpb, gch, lds, st); break;
    case 8: ok = conv_pw_run_ks8(p, ep, ops, rpb, gch, lds, st); break;
    case -1: ok = conv_pw_run_ks1_w4(p, ep, ops, rpb, gch, lds, st); break;
    case -2: ok = conv_pw_run_ks2_w4(p, ep, ops, rpb, gch, lds, st); break;
    case -4: ok = conv_pw_run_ks4_w4(p, ep, ops, rpb, gch, lds, st); break;
    default: ok = conv_pw_run_ks8_w4(p, ep, ops, rpb, gch, lds, st); break;
  }
  if (!ok) {
    char msg[128];
    snprintf(msg, sizeof msg, "pointwise conv: no kernel for backward-BN epilogue operand set 0x%x", ops);
    throw std::runtime_error(msg);
  }
}

PVA_NS_END  // namespace PVA_NS
