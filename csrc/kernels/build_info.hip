// Build provenance of liboni_hip.so: the content hash of csrc/kernels/* it was compiled from
// (oni355/utils/provenance.py; checked when the package loads the library).
#include "oni_common.h"

#ifndef ONI_SRC_HASH
#define ONI_SRC_HASH "unknown"
#endif

ONI_API const char* oni_hip_src_hash() { return ONI_SRC_HASH; }
