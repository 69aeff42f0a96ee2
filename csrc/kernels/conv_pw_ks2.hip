// Instantiations of the pointwise conv kernel (conv_pw_impl.h) for K <= 64 (KS = 2 MFMA k-steps).
#include "conv_pw_impl.h"

PVA_NS_BEGIN

bool conv_pw_run_ks2(const ConvParams& p, int ep, int ops, int rpb, int gch, size_t lds, hipStream_t st) {
  return launch_ks<2, 8>(p, ep, ops, rpb, gch, lds, st);
}

PVA_NS_END  // namespace PVA_NS
