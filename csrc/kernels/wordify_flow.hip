// K02+K03 -- netflow featurization: order keys for the three binned columns, then the fused
// bin-lookup + port rule + word packing (one thread per flow, two 32-bit word keys out).
//
// Behaviour spec: SURVEY.md §2.8 "Flow" (oni-ml FlowWordCreation, [U-M]): the reference builds
// the string  [-1_]<port>_<timeBin>_<ibytBin>_<ipktBin>  per endpoint; here the same information
// is bit-packed so the GPU never touches strings (strings are rendered only for CSV output):
//
//   bit 28      : direction flag ("-1_" prefix)
//   bits 11..27 : port code (0..65535, 65536 = "111111", 65537 = "333333")
//   bits  7..10 : time bin  (deciles of hour + min/60 + sec/3600)
//   bits  3..6  : ibyt bin  (deciles)
//   bits  0..2  : ipkt bin  (quintiles)
#include "oni_common.h"

namespace {

constexpr uint32_t kPort111111 = 65536u, kPort333333 = 65537u;

__global__ void k_flow_keys(const int32_t* __restrict__ hour, const int32_t* __restrict__ minute,
                            const int32_t* __restrict__ second, const int64_t* __restrict__ ibyt,
                            const int64_t* __restrict__ ipkt, int64_t n, uint32_t* __restrict__ tkey,
                            uint32_t* __restrict__ bkey, uint32_t* __restrict__ pkey) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float t = ((float)hour[i] + (float)minute[i] / 60.0f) + (float)second[i] / 3600.0f;
    tkey[i] = oni::f32_key(t);
    const int64_t b = ibyt[i], p = ipkt[i];
    bkey[i] = b <= 0 ? 0u : (b >= 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)b);
    pkey[i] = p <= 0 ? 0u : (p >= 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)p);
  }
}

__device__ __forceinline__ uint32_t bin_of(uint32_t k, const uint32_t* cuts, int nc) {
  uint32_t b = 0;
  for (int c = 0; c < nc; ++c) b += k > cuts[c];
  return b;
}

// cuts layout: [0..nt) time cuts, [nt..nt+nb) ibyt cuts, [nt+nb..nt+nb+np) ipkt cuts
__global__ __launch_bounds__(256) void k_flow_wordify(const int32_t* __restrict__ sport,
                                                      const int32_t* __restrict__ dport,
                                                      const uint32_t* __restrict__ tkey,
                                                      const uint32_t* __restrict__ bkey,
                                                      const uint32_t* __restrict__ pkey, int64_t n,
                                                      const uint32_t* __restrict__ cuts, int nt, int nb, int np,
                                                      uint32_t* __restrict__ src_word,
                                                      uint32_t* __restrict__ dst_word) {
  __shared__ uint32_t sc[32];
  if (threadIdx.x < nt + nb + np) sc[threadIdx.x] = cuts[threadIdx.x];
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t tb = bin_of(tkey[i], sc, nt);
    const uint32_t bb = bin_of(bkey[i], sc + nt, nb);
    const uint32_t pb = bin_of(pkey[i], sc + nt + nb, np);
    const int32_t sp = sport[i], dp = dport[i];
    uint32_t port, sdir = 0, ddir = 0;
    if (sp == 0 && dp == 0) {
      port = 0;
    } else if (dp == 0 && sp > 0) {
      port = (uint32_t)sp; sdir = 1;
    } else if (sp == 0 && dp > 0) {
      port = (uint32_t)dp; ddir = 1;
    } else if (sp <= 1024 && dp <= 1024) {
      port = kPort111111;
    } else if (sp <= 1024 && dp > 1024) {
      port = (uint32_t)sp; sdir = 1;
    } else if (sp > 1024 && dp <= 1024) {
      port = (uint32_t)dp; ddir = 1;
    } else {
      port = kPort333333;
    }
    const uint32_t base = (port << 11) | (tb << 7) | (bb << 3) | pb;
    src_word[i] = base | (sdir << 28);
    dst_word[i] = base | (ddir << 28);
  }
}

}  // namespace

ONI_API int oni_flow_keys(const int32_t* hour, const int32_t* minute, const int32_t* second, const int64_t* ibyt,
                          const int64_t* ipkt, int64_t n, uint32_t* tkey, uint32_t* bkey, uint32_t* pkey,
                          hipStream_t s) {
  k_flow_keys<<<oni::grid_for(n), 256, 0, s>>>(hour, minute, second, ibyt, ipkt, n, tkey, bkey, pkey);
  return (int)hipGetLastError();
}

ONI_API int oni_flow_wordify(const int32_t* sport, const int32_t* dport, const uint32_t* tkey, const uint32_t* bkey,
                             const uint32_t* pkey, int64_t n, const uint32_t* cuts, int nt, int nb, int np,
                             uint32_t* src_word, uint32_t* dst_word, hipStream_t s) {
  if (nt + nb + np > 32 || nt > 15 || nb > 15 || np > 7) return (int)hipErrorInvalidValue;
  k_flow_wordify<<<oni::grid_for(n), 256, 0, s>>>(sport, dport, tkey, bkey, pkey, n, cuts, nt, nb, np, src_word,
                                                  dst_word);
  return (int)hipGetLastError();
}
