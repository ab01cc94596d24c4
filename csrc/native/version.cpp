#include "oni_native.h"

ONI_NATIVE_API int oni_native_version() { return 1; }

#ifndef ONI_SRC_HASH
#define ONI_SRC_HASH "unknown"
#endif

// content hash of the host sources this library was built from (oni355/utils/provenance.py)
ONI_NATIVE_API const char* oni_native_src_hash() { return ONI_SRC_HASH; }
