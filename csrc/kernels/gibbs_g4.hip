// Instantiations of the Gibbs sweep kernels for four-lane units (K = 57..112) (see gibbs_sampler.h).
#include "gibbs_sampler.h"

int oni_gibbs_dispatch_g4(const OniGibbs& a, int KP, bool init, int mode, int qpf, hipStream_t s) {
#define ONI_CASE(g_, kp_) \
  if (KP == kp_) return launch_gibbs<g_, kp_>(a, init, mode, qpf, s);
  ONI_CASE(4, 8) ONI_CASE(4, 12) ONI_CASE(4, 16) ONI_CASE(4, 20) ONI_CASE(4, 24) ONI_CASE(4, 28)
#undef ONI_CASE
  return (int)hipErrorInvalidValue;
}
