// oni355 host runtime (C++17): decoders, lda-c compatible VEM engine, formatters.
// Exported through a plain C ABI and loaded with ctypes (oni355/ops/native.py).
#pragma once
#include <cstddef>
#include <cstdint>

#define ONI_NATIVE_API extern "C" __attribute__((visibility("default")))
