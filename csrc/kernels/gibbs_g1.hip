// Instantiations of the Gibbs sweep kernels for one-lane units (K ≤ 32) (see gibbs_sampler.h).
#include "gibbs_sampler.h"

int oni_gibbs_dispatch_g1(const OniGibbs& a, int KP, bool init, int mode, int qpf, hipStream_t s) {
#define ONI_CASE(g_, kp_) \
  if (KP == kp_) return launch_gibbs<g_, kp_>(a, init, mode, qpf, s);
  ONI_CASE(1, 4) ONI_CASE(1, 8) ONI_CASE(1, 12) ONI_CASE(1, 16) ONI_CASE(1, 20) ONI_CASE(1, 24) ONI_CASE(1, 28)
  ONI_CASE(1, 32)
#undef ONI_CASE
  return (int)hipErrorInvalidValue;
}
