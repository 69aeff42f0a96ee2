// Instantiations of the pointwise conv kernel (conv_pw_impl.h) for K <= 128 (KS = 4 MFMA k-steps), 4-wave workgroups (cfg bit 3).
#include "conv_pw_impl.h"

PVA_NS_BEGIN

bool conv_pw_run_ks4_w4(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st) {
  return launch_ks<4, 4>(p, ep, ops, rpb, gch, lds, st);
}

PVA_NS_END  // namespace PVA_NS
