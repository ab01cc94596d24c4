// K15/K16 -- per-event suspiciousness scores + threshold/top-N selection.
//
// Reference behaviour (oni-ml FlowPostLDA / DNSPostLDA / ProxyPostLDA, SURVEY.md §2.2 C24, [U-H]):
// score(event) = Σ_k θ[doc,k]·φ[word,k]; flows take min over (src IP, src word) and (dst IP,
// dst word); keep score < TOL, sort ascending, first MAXRESULTS.
//
// Here: one thread per event, θ/φ rows gathered with 16-B vector loads (rows padded to KS, pads
// are zero) and dotted in fixed k order (pinned numerics, no fma contraction). The same pass
// builds an LDS histogram of the top 11 bits of the score's order key for the events under TOL,
// so the MAXRESULTS-th smallest score's bucket is known without sorting N scores; a compaction
// pass then keeps only that bucket prefix (usually ~MAXRESULTS events) for a tiny final sort.
#include "oni_common.h"

namespace {

template <int KS>
__device__ __forceinline__ float dot_rows(const float* __restrict__ a, const float* __restrict__ b) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < KS; j += 4) {
    const float4 x = *reinterpret_cast<const float4*>(a + j);
    const float4 y = *reinterpret_cast<const float4*>(b + j);
    s = s + x.x * y.x;
    s = s + x.y * y.y;
    s = s + x.z * y.z;
    s = s + x.w * y.w;
  }
  return s;
}

__device__ __forceinline__ float dot_rows_dyn(const float* __restrict__ a, const float* __restrict__ b, int KS) {
  float s = 0.f;
  for (int j = 0; j < KS; j += 4) {
    const float4 x = *reinterpret_cast<const float4*>(a + j);
    const float4 y = *reinterpret_cast<const float4*>(b + j);
    s = s + x.x * y.x;
    s = s + x.y * y.y;
    s = s + x.z * y.z;
    s = s + x.w * y.w;
  }
  return s;
}

template <int KS>
__global__ __launch_bounds__(256) void k_score(const float* __restrict__ theta, const float* __restrict__ phi,
                                                int ks_dyn, const int32_t* __restrict__ d1,
                                                const int32_t* __restrict__ w1, const int32_t* __restrict__ d2,
                                                const int32_t* __restrict__ w2, int64_t n, float tol,
                                                float* __restrict__ out, float* __restrict__ out1,
                                                float* __restrict__ out2, uint32_t* __restrict__ hist) {
  __shared__ uint32_t lh[2048];
  if (hist) {
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) lh[i] = 0u;
    __syncthreads();
  }
  const int ks = KS > 0 ? KS : ks_dyn;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float* t1 = theta + (int64_t)d1[i] * ks;
    const float* p1 = phi + (int64_t)w1[i] * ks;
    const float s1 = KS > 0 ? dot_rows<(KS > 0 ? KS : 4)>(t1, p1) : dot_rows_dyn(t1, p1, ks);
    float sc = s1;
    if (d2) {
      const float* t2 = theta + (int64_t)d2[i] * ks;
      const float* p2 = phi + (int64_t)w2[i] * ks;
      const float s2 = KS > 0 ? dot_rows<(KS > 0 ? KS : 4)>(t2, p2) : dot_rows_dyn(t2, p2, ks);
      sc = s2 < s1 ? s2 : s1;
      if (out2) out2[i] = s2;
    }
    if (out1) out1[i] = s1;
    out[i] = sc;
    if (hist && sc < tol) atomicAdd(&lh[oni::f32_key(sc) >> 21], 1u);
  }
  if (hist) {
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) {
      const uint32_t v = lh[i];
      if (v) atomicAdd(&hist[i], v);
    }
  }
}

// Keep events with score < tol and order-key bucket ≤ bmax; wave-aggregated slot allocation.
__global__ __launch_bounds__(256) void k_select(const float* __restrict__ score, int64_t n, float tol, uint32_t bmax,
                                                 uint32_t* __restrict__ count, int64_t* __restrict__ out_idx,
                                                 float* __restrict__ out_score, int64_t cap) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n_iter = (n + stride - 1) / stride;
  for (int64_t it = 0; it < n_iter; ++it) {
    const int64_t i = it * stride + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool keep = false;
    float sc = 0.f;
    if (i < n) {
      sc = score[i];
      keep = sc < tol && (oni::f32_key(sc) >> 21) <= bmax;
    }
    const uint64_t m = __ballot(keep);
    if (m == 0) continue;
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (oni::lane_id() == leader) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    if (keep) {
      const uint32_t slot = base + (uint32_t)__popcll(m & ((1ull << oni::lane_id()) - 1ull));
      if ((int64_t)slot < cap) {
        out_idx[slot] = i;
        out_score[slot] = sc;
      }
    }
  }
}

// ---- pair-plan scoring (SURVEY.md §2.6 K15 "baseline": SDDMM over unique pairs) -------------
// Events repeat (doc, word) pairs heavily (12.5M synthetic flows → 25M endpoint tokens but only
// 2.7M distinct pairs), and a per-event θ-row gather is a random 80-B read from a table that does
// not fit an XCD's L2. So: score each distinct pair once (pairs are doc-major, so consecutive
// lanes reuse the same θ row), then every event gathers two 4-B pair scores. Same dot order as
// k_score → bitwise-identical scores.
template <int KS>
__global__ __launch_bounds__(256) void k_pair_score(const float* __restrict__ theta, const float* __restrict__ phi,
                                                     int ks_dyn, const int32_t* __restrict__ pdoc,
                                                     const int32_t* __restrict__ pword, int64_t P,
                                                     float* __restrict__ ps) {
  const int ks = KS > 0 ? KS : ks_dyn;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += stride) {
    const float* t = theta + (int64_t)pdoc[i] * ks;
    const float* f = phi + (int64_t)pword[i] * ks;
    ps[i] = KS > 0 ? dot_rows<(KS > 0 ? KS : 4)>(t, f) : dot_rows_dyn(t, f, ks);
  }
}

// event score = ps[p1] (or min(ps[p1], ps[p2]) for two-endpoint events) + the order-key histogram
// of scores under tol, aggregated per wave before the LDS atomics (equal buckets are common).
__global__ __launch_bounds__(256) void k_event_min(const float* __restrict__ ps, const int32_t* __restrict__ p1,
                                                    const int32_t* __restrict__ p2, int64_t n, float tol,
                                                    float* __restrict__ out, float* __restrict__ out1,
                                                    float* __restrict__ out2, uint32_t* __restrict__ hist) {
  __shared__ uint32_t lh[2048];
  if (hist) {
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) lh[i] = 0u;
    __syncthreads();
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n_iter = (n + stride - 1) / stride;
  for (int64_t it = 0; it < n_iter; ++it) {
    const int64_t i = it * stride + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool in = i < n;
    float sc = 0.f;
    if (in) {
      const float s1 = ps[p1[i]];
      sc = s1;
      if (p2) {
        const float s2 = ps[p2[i]];
        sc = s2 < s1 ? s2 : s1;
        if (out2) out2[i] = s2;
      }
      if (out1) out1[i] = s1;
      out[i] = sc;
    }
    // one LDS atomic per lane: the LDS serializes same-bucket lanes in hardware; a wave-aggregation
    // loop (ballot/shfl per distinct bucket) measured ~250 VALU instructions per wave-iteration
    // here (scores spread over tens of buckets) and made this gather kernel VALU-bound
    if (hist && in && sc < tol) atomicAdd(&lh[oni::f32_key(sc) >> 21], 1u);
  }
  if (hist) {
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) {
      const uint32_t v = lh[i];
      if (v) atomicAdd(&hist[i], v);
    }
  }
}

}  // namespace

ONI_API int oni_score(const float* theta, const float* phi, int KS, const int32_t* d1, const int32_t* w1,
                      const int32_t* d2, const int32_t* w2, int64_t n, float tol, float* out, float* out1,
                      float* out2, uint32_t* hist, hipStream_t s) {
  if (KS % 4 != 0) return (int)hipErrorInvalidValue;
  const unsigned grid = oni::grid_for(n, 256, 2048);
#define ONI_S(k_) \
  if (KS == k_) { k_score<k_><<<grid, 256, 0, s>>>(theta, phi, KS, d1, w1, d2, w2, n, tol, out, out1, out2, hist); \
                  return (int)hipGetLastError(); }
  ONI_S(20) ONI_S(24) ONI_S(32) ONI_S(52) ONI_S(64) ONI_S(100) ONI_S(104) ONI_S(128)
#undef ONI_S
  k_score<0><<<grid, 256, 0, s>>>(theta, phi, KS, d1, w1, d2, w2, n, tol, out, out1, out2, hist);
  return (int)hipGetLastError();
}

ONI_API int oni_select_below(const float* score, int64_t n, float tol, uint32_t bmax, uint32_t* count,
                             int64_t* out_idx, float* out_score, int64_t cap, hipStream_t s) {
  k_select<<<oni::grid_for(n, 256, 2048), 256, 0, s>>>(score, n, tol, bmax, count, out_idx, out_score, cap);
  return (int)hipGetLastError();
}

ONI_API int oni_pair_score(const float* theta, const float* phi, int KS, const int32_t* pdoc, const int32_t* pword,
                           int64_t P, float* ps, hipStream_t s) {
  if (KS % 4 != 0) return (int)hipErrorInvalidValue;
  if (P == 0) return 0;
  const unsigned grid = oni::grid_for(P, 256, 4096);
#define ONI_P(k_) \
  if (KS == k_) { k_pair_score<k_><<<grid, 256, 0, s>>>(theta, phi, KS, pdoc, pword, P, ps); \
                  return (int)hipGetLastError(); }
  ONI_P(20) ONI_P(24) ONI_P(32) ONI_P(52) ONI_P(64) ONI_P(100) ONI_P(104) ONI_P(128)
#undef ONI_P
  k_pair_score<0><<<grid, 256, 0, s>>>(theta, phi, KS, pdoc, pword, P, ps);
  return (int)hipGetLastError();
}

ONI_API int oni_event_min(const float* ps, const int32_t* p1, const int32_t* p2, int64_t n, float tol, float* out,
                          float* out1, float* out2, uint32_t* hist, hipStream_t s) {
  if (n == 0) return 0;
  k_event_min<<<oni::grid_for(n, 256, 2048), 256, 0, s>>>(ps, p1, p2, n, tol, out, out1, out2, hist);
  return (int)hipGetLastError();
}
