#include "oni_native.h"

ONI_NATIVE_API int oni_native_version() { return 1; }
