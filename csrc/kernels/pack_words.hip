// K05/K06 -- table-driven word packing for DNS and proxy events.
//
// A word is a fixed-width integer with one bit-field per component (SURVEY.md §2.8 packing
// decision): binned components (bin(key) = #{cuts < key}, cuts in LDS) and raw categorical
// fields (masked). The field table (shifts, masks, cut lists) comes from the Python spec
// (oni355/pipeline/dns.py, proxy.py), so the word layout is data, not code.
#include "oni_common.h"

constexpr int kMaxBinned = 8;
constexpr int kMaxRaw = 4;
constexpr int kMaxCuts = 15;

struct OniPack {
  const uint32_t* key[kMaxBinned];  // order keys per binned component
  int32_t ncuts[kMaxBinned];
  int32_t kshift[kMaxBinned];
  uint32_t cuts[kMaxBinned][kMaxCuts];
  const int32_t* raw[kMaxRaw];      // raw categorical components (int32)
  uint32_t rmask[kMaxRaw];
  int32_t rshift[kMaxRaw];
  const uint8_t* raw8;              // optional u8 component (e.g. top-domain flag)
  uint32_t r8mask;
  int32_t r8shift;
  int32_t nkeys, nraw;
  int64_t n;
  uint64_t* out;
  const uint32_t* dcuts;            // optional: the cut lists on the device, concatenated in component
                                    // order (ncuts[f] each; e.g. straight from the device quantile
                                    // select) -- then ``cuts`` is ignored
};

namespace {

__global__ __launch_bounds__(256) void k_pack(const OniPack a) {
  __shared__ uint32_t sc[kMaxBinned][kMaxCuts];
  if (a.dcuts) {
    int off = 0;
    for (int f = 0; f < a.nkeys; ++f) {
      for (int c = threadIdx.x; c < a.ncuts[f]; c += blockDim.x) sc[f][c] = a.dcuts[off + c];
      off += a.ncuts[f];
    }
  } else {
    for (int i = threadIdx.x; i < kMaxBinned * kMaxCuts; i += blockDim.x)
      sc[i / kMaxCuts][i % kMaxCuts] = a.cuts[i / kMaxCuts][i % kMaxCuts];
  }
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    uint64_t w = 0;
    for (int f = 0; f < a.nkeys; ++f) {
      const uint32_t k = a.key[f][i];
      uint32_t b = 0;
      for (int c = 0; c < a.ncuts[f]; ++c) b += k > sc[f][c];
      w |= (uint64_t)b << a.kshift[f];
    }
    for (int f = 0; f < a.nraw; ++f) w |= (uint64_t)((uint32_t)a.raw[f][i] & a.rmask[f]) << a.rshift[f];
    if (a.raw8) w |= (uint64_t)(a.raw8[i] & a.r8mask) << a.r8shift;
    a.out[i] = w;
  }
}

}  // namespace

ONI_API int oni_pack_sizeof() { return (int)sizeof(OniPack); }

ONI_API int oni_pack_words(const OniPack* a, hipStream_t s) {
  if (a->nkeys > kMaxBinned || a->nraw > kMaxRaw) return (int)hipErrorInvalidValue;
  for (int f = 0; f < a->nkeys; ++f)
    if (a->ncuts[f] > kMaxCuts) return (int)hipErrorInvalidValue;
  if (a->n == 0) return 0;
  k_pack<<<oni::grid_for(a->n), 256, 0, s>>>(*a);
  return (int)hipGetLastError();
}
