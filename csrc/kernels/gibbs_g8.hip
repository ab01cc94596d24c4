// Instantiations of the Gibbs sweep kernels for 8- and 16-lane units (K > 112, ONI_TILING=narrow) (see gibbs_sampler.h).
#include "gibbs_sampler.h"

int oni_gibbs_dispatch_g8(const OniGibbs& a, int G, int KP, bool init, int mode, int qpf, hipStream_t s) {
#define ONI_CASE(g_, kp_) \
  if (G == g_ && KP == kp_) return launch_gibbs<g_, kp_>(a, init, mode, qpf, s);
  ONI_CASE(8, 8) ONI_CASE(8, 12) ONI_CASE(8, 16)
  ONI_CASE(16, 8) ONI_CASE(16, 16)
#undef ONI_CASE
  return (int)hipErrorInvalidValue;
}
