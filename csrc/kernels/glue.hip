// Small fused glue ops of the day path: each replaces a chain of torch
// elementwise kernels (cat → int64 conversion → mask) with one pass over the inputs.
#include "oni_common.h"

namespace {

// out[0:n) = zero-extended a, out[n:2n) = zero-extended b (u32 bits held in int32 tensors): the
// day's doc keys (sip ‖ dip) and word keys (src word ‖ dst word) as non-negative int64 in one
// launch instead of torch.cat + .to(int64) + & 0xFFFFFFFF (three kernels, two temporaries).
__global__ __launch_bounds__(256) void k_widen_pair(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                                    int64_t n, uint64_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    out[i] = (uint64_t)a[i];
    out[n + i] = (uint64_t)b[i];
  }
}

}  // namespace

ONI_API int oni_widen_pair(const uint32_t* a, const uint32_t* b, int64_t n, uint64_t* out, hipStream_t s) {
  if (n <= 0) return 0;
  k_widen_pair<<<oni::grid_for(n, 256, 8192), 256, 0, s>>>(a, b, n, out);
  return (int)hipGetLastError();
}
