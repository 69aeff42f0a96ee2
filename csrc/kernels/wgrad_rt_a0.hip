// Instantiations of the row-table weight-gradient kernel (wgrad_rt_impl.h), AFF = 0.
#include "wgrad_rt_impl.h"

PVA_NS_BEGIN

void wgrad_rt_run_a0(int v, bool bp64, bool check, const wgrad_rt::RtParams& rp, hipStream_t st) {
  wgrad_rt::launch_aff<false>(v, bp64, check, rp, st);
}

PVA_NS_END  // namespace PVA_NS
