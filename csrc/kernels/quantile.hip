// K01 -- exact multi-quantile cut points by LSD-free radix *select* (no sort).
//
// Replaces the reference's Spark `sortBy` ECDF (oni-ml Quantiles.computeDeciles / computeQuintiles,
// SURVEY.md §2.2 C15, [U-M]) with three histogram passes over u32 order keys (11+11+10 bits).
// Every quantile q carries its own radix prefix; a pass histograms only the keys whose high bits
// match one of the (de-duplicated) live prefixes, all of them in ONE read of the column, into
// P×2^nbits LDS bins. Per-block bins are flushed to the global histogram with integer atomics on
// non-zero bins only. The host picks the digit holding each target rank between passes (and, for
// data-parallel runs, all-reduces the histograms over RCCL first: collective X03).
#include "oni_common.h"

namespace {

constexpr int kMaxPrefixes = 16;

template <int NBITS>
__global__ __launch_bounds__(256) void k_radix_hist(const uint32_t* __restrict__ keys, int64_t n, int shift,
                                                     const uint32_t* __restrict__ prefixes, int P,
                                                     uint32_t mask, uint32_t* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lh[];
  constexpr int B = 1 << NBITS;
  const int nb = P * B;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) lh[i] = 0u;
  uint32_t pre[kMaxPrefixes];
#pragma unroll
  for (int p = 0; p < kMaxPrefixes; ++p) pre[p] = p < P ? prefixes[p] : 0xFFFFFFFFu;
  __syncthreads();
  // Skewed columns (most flows of 1 packet, ...) put most lanes of a wave on ONE bin, and
  // same-address LDS atomics serialise: for the key's first matching prefix, the lanes sharing the
  // first active lane's bin add their count with one atomic. (The device-only pipeline's prefixes
  // are not de-duplicated: a key adds to every prefix it matches, the later ones one by one.)
  auto count = [&](uint32_t k) {
    const uint32_t hi = k & mask;
    const int digit = (int)((k >> shift) & (B - 1));
    int bin = -1;
#pragma unroll
    for (int p = 0; p < kMaxPrefixes; ++p) {
      if (p < P && hi == pre[p]) {
        if (bin < 0) bin = p * B + digit;
        else atomicAdd(&lh[p * B + digit], 1u);
      }
    }
    const int b0 = __builtin_amdgcn_readfirstlane(bin);
    const uint64_t same = __ballot(bin == b0);
    if (bin == b0) {
      if (b0 >= 0 && __lane_id() == __ffsll((unsigned long long)same) - 1)
        atomicAdd(&lh[b0], (uint32_t)__popcll(same));
    } else if (bin >= 0) {
      atomicAdd(&lh[bin], 1u);
    }
  };
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i0 = 0;
  if ((reinterpret_cast<uintptr_t>(keys) & 15u) == 0) {
    // four keys per 16-B load: four independent loads in flight per lane, not one
    const int64_t n4 = n / 4;
    const uint4* k4 = reinterpret_cast<const uint4*>(keys);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
      const uint4 v = k4[i];
      count(v.x);
      count(v.y);
      count(v.z);
      count(v.w);
    }
    i0 = n4 * 4;
  }
  for (int64_t i = i0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) count(keys[i]);
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    const uint32_t v = lh[i];
    if (v) atomicAdd(&hist[i], v);
  }
}

__global__ void k_f32_keys(const float* __restrict__ x, int64_t n, uint32_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = oni::f32_key(x[i]);
}

__global__ void k_i64_keys(const int64_t* __restrict__ x, int64_t n, uint32_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t v = x[i];
    out[i] = v <= 0 ? 0u : (v >= 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)v);
  }
}

// bin(x) = #{cuts c : key(x) > c}; one thread per element, cuts in scalar registers.
__global__ void k_bin_keys(const uint32_t* __restrict__ keys, int64_t n, const uint32_t* __restrict__ cuts, int nc,
                           uint8_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t k = keys[i];
    int b = 0;
    for (int c = 0; c < nc; ++c) b += k > cuts[c];
    out[i] = (uint8_t)b;
  }
}

// Device-side radix-select step (no host round trip between passes): wave q scans query q's
// histogram (pass 1: the feature's single histogram, all prefixes being 0) for the first digit
// whose cumulative count exceeds the query's remaining rank -- searchsorted(cumsum, rank, right)
// capped at B-1, exactly the host step it replaces -- and narrows the prefix / rank. Each lane
// owns B/64 consecutive bins: lane sums, one wave prefix scan, then the owning lane walks its bins.
__global__ __launch_bounds__(64) void k_quantile_pick(const uint32_t* __restrict__ hist,
                                                      const int32_t* __restrict__ base, int nq, int B, int shift,
                                                      uint32_t* __restrict__ prefix, int64_t* __restrict__ rank) {
  const int q = blockIdx.x;
  const int lane = threadIdx.x;
  if (q >= nq) return;
  const uint32_t* h = hist + base[q];
  const int per = B / oni::kWave;
  const int64_t r = rank[q];
  int64_t mine = 0;
  for (int j = 0; j < per; ++j) mine += h[lane * per + j];
  int64_t incl = mine;  // inclusive scan over lanes
#pragma unroll
  for (int d = 1; d < oni::kWave; d <<= 1) {
    const int64_t y = __shfl_up(incl, d);
    if (lane >= d) incl += y;
  }
  const int64_t excl = incl - mine;
  // the lane whose bins hold the first cumulative count > r (none: digit B-1)
  const uint64_t hit = __ballot(incl > r);
  if (hit) {
    const int owner = __ffsll((unsigned long long)hit) - 1;
    if (lane == owner) {
      int64_t cum = excl;
      int digit = lane * per + per - 1;
      int64_t below = cum;
      for (int j = 0; j < per; ++j) {
        const int64_t nxt = cum + h[lane * per + j];
        if (nxt > r) {
          digit = lane * per + j;
          below = cum;
          break;
        }
        cum = nxt;
      }
      if (digit > 0) rank[q] = r - below;
      prefix[q] |= (uint32_t)digit << shift;
    }
  } else if (lane == oni::kWave - 1) {
    // every count ≤ r: digit B-1, rank -= cumsum[B-2]
    const int64_t below = incl - h[B - 1];
    rank[q] = r - below;
    prefix[q] |= (uint32_t)(B - 1) << shift;
  }
}

}  // namespace

ONI_API int oni_quantile_pick(const uint32_t* hist, const int32_t* base, int nq, int nbits, int shift, uint32_t* prefix,
                              int64_t* rank, hipStream_t s) {
  if (nq < 1 || nbits < 1 || nbits > 16) return (int)hipErrorInvalidValue;
  if ((1 << nbits) % 64) return (int)hipErrorInvalidValue;
  k_quantile_pick<<<nq, 64, 0, s>>>(hist, base, nq, 1 << nbits, shift, prefix, rank);
  return (int)hipGetLastError();
}

ONI_API int oni_radix_hist(const uint32_t* keys, int64_t n, int shift, int nbits, const uint32_t* prefixes, int P,
                           uint32_t mask, uint32_t* hist, hipStream_t s) {
  if (P < 1 || P > kMaxPrefixes) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)P << nbits << 2;
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  // 2048 workgroups (8 per CU): the loop is latency-bound, 512 left 8 waves per CU
  const unsigned grid = oni::grid_for((n + 3) / 4, 256, 2048);
  if (nbits == 11)
    k_radix_hist<11><<<grid, 256, lds, s>>>(keys, n, shift, prefixes, P, mask, hist);
  else if (nbits == 10)
    k_radix_hist<10><<<grid, 256, lds, s>>>(keys, n, shift, prefixes, P, mask, hist);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

ONI_API int oni_f32_keys(const float* x, int64_t n, uint32_t* out, hipStream_t s) {
  k_f32_keys<<<oni::grid_for(n), 256, 0, s>>>(x, n, out);
  return (int)hipGetLastError();
}

ONI_API int oni_i64_keys(const int64_t* x, int64_t n, uint32_t* out, hipStream_t s) {
  k_i64_keys<<<oni::grid_for(n), 256, 0, s>>>(x, n, out);
  return (int)hipGetLastError();
}

ONI_API int oni_bin_keys(const uint32_t* keys, int64_t n, const uint32_t* cuts, int nc, uint8_t* out, hipStream_t s) {
  k_bin_keys<<<oni::grid_for(n), 256, 0, s>>>(keys, n, cuts, nc, out);
  return (int)hipGetLastError();
}
