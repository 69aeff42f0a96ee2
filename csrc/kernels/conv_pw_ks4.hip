// Instantiations of the pointwise conv kernel (conv_pw_impl.h) for K <= 128 (KS = 4 MFMA k-steps).
#include "conv_pw_impl.h"

PVA_NS_BEGIN

bool conv_pw_run_ks4(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st) {
  return launch_ks<4, 8>(p, ep, ops, rpb, gch, lds, st);
}

PVA_NS_END  // namespace PVA_NS
