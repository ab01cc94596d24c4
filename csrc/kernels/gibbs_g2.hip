// Instantiations of the Gibbs sweep kernels for two-lane units (K = 33..56) (see gibbs_sampler.h).
#include "gibbs_sampler.h"

int oni_gibbs_dispatch_g2(const OniGibbs& a, int KP, bool init, int mode, int qpf, hipStream_t s) {
#define ONI_CASE(g_, kp_) \
  if (KP == kp_) return launch_gibbs<g_, kp_>(a, init, mode, qpf, s);
  ONI_CASE(2, 20) ONI_CASE(2, 24) ONI_CASE(2, 28)
#undef ONI_CASE
  return (int)hipErrorInvalidValue;
}
