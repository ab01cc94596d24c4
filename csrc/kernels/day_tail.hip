// The tail of a training run (K13/K14 + the numerical health check) in a few launches instead of
// ~30 small torch kernels with a host round trip between many of them (profiles/r3: ~1.6 ms of
// a 65 ms flow day was the gaps between those kernels, not their work).
//
//  * k_tail_partials / k_tail_final: one pass over n_wk, q, n_k and n_dk giving, per block, the
//    collapsed log-likelihood's lgamma sums (Griffiths & Steyvers 2004) and the health flags
//    (non-finite q entries, negative counts); a single-block kernel reduces the per-block
//    partials in a fixed order, so the value is deterministic (same inputs, same bits).
//  * k_theta_rows / k_phi_rows: θ = (n_dk + a)/(n_d + a_K) and φ = (n_wk + b)/(n_k + b_V) in f32
//    from (averaged) counts, the exact expressions the torch path evaluated (oni355/models/gibbs.py).
#include "oni_common.h"

namespace {

constexpr int kTailBlock = 256;
constexpr int kTailVals = 8;  // [Σlgamma(n_wk+β), Σlgamma(n_k+Vβ), Σlgamma(n_dk+α), Σlgamma(n_d+Kα),
                              //  #non-finite q, #negative n_wk/n_k, #negative n_dk, unused]

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int m = 1; m < oni::kWave; m <<= 1) v += __shfl_xor(v, m);
  return v;
}

__global__ __launch_bounds__(kTailBlock) void k_tail_partials(const int32_t* __restrict__ nwk,
                                                              const float* __restrict__ q,
                                                              const int32_t* __restrict__ nk,
                                                              const int32_t* __restrict__ ndk, int64_t V, int64_t D,
                                                              int K, int KS, double alpha, double beta, double vbeta,
                                                              double kalpha, double* __restrict__ part) {
  double acc[kTailVals];
#pragma unroll
  for (int j = 0; j < kTailVals; ++j) acc[j] = 0.0;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t VK = V * K;
  for (int64_t i = tid; i < VK; i += stride) {
    const int64_t w = i / K;
    const int k = (int)(i - w * K);
    const int32_t n = nwk[w * KS + k];
    const float qv = q[w * KS + k];
    acc[0] += lgamma((double)n + beta);
    acc[4] += isfinite(qv) ? 0.0 : 1.0;
    acc[5] += n < 0 ? 1.0 : 0.0;
  }
  if (blockIdx.x == 0)
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
      acc[1] += lgamma((double)nk[k] + vbeta);
      acc[5] += nk[k] < 0 ? 1.0 : 0.0;
    }
  for (int64_t d = tid; d < D; d += stride) {
    const int32_t* r = ndk + d * KS;
    int64_t nd = 0;
    for (int k = 0; k < K; ++k) {
      const int32_t n = r[k];
      nd += n;
      acc[2] += lgamma((double)n + alpha);
      acc[6] += n < 0 ? 1.0 : 0.0;
    }
    acc[3] += lgamma((double)nd + kalpha);
  }
  __shared__ double red[kTailBlock / oni::kWave][kTailVals];
  const int wave = threadIdx.x / oni::kWave, lane = threadIdx.x % oni::kWave;
#pragma unroll
  for (int j = 0; j < kTailVals; ++j) {
    const double v = wave_sum_d(acc[j]);
    if (lane == 0) red[wave][j] = v;
  }
  __syncthreads();
  if (threadIdx.x < kTailVals) {
    double v = 0.0;
    for (int w = 0; w < kTailBlock / oni::kWave; ++w) v += red[w][threadIdx.x];
    part[(int64_t)blockIdx.x * kTailVals + threadIdx.x] = v;
  }
}

// wave j reduces value j over the blocks: lane-strided sums, then the butterfly (a fixed order:
// deterministic)
__global__ __launch_bounds__(kTailVals * 64) void k_tail_final(const double* __restrict__ part, int nblocks,
                                                              double* __restrict__ out) {
  const int j = threadIdx.x / oni::kWave, lane = threadIdx.x % oni::kWave;
  double v = 0.0;
  for (int b = lane; b < nblocks; b += oni::kWave) v += part[(int64_t)b * kTailVals + j];
  v = wave_sum_d(v);
  if (lane == 0) out[j] = v;
}

// 256 rows per block: thread t sums row t's counts in int64 (exact for any document: averaged
// posterior counts are S times a document's length and pass 2^24 for heavy IPs) and rounds the
// sum to f32 once, into LDS, then the block reads and writes its rows' KS columns
// coalesced (a row per thread touched KS scattered words per lane).
// Count type C: int32 for one sample's counts, int64 for the posterior-average sums (S samples of
// counts up to 2^31 each: an int32 sum wraps once a count passes 2^31 / S).
template <typename C>
__global__ __launch_bounds__(256) void k_theta_rows(const C* __restrict__ n, int64_t D, int K, int KS, float add,
                                                    float den_add, float* __restrict__ th) {
  __shared__ float den[256];
  for (int64_t r0 = (int64_t)blockIdx.x * 256; r0 < D; r0 += (int64_t)gridDim.x * 256) {
    const int64_t d = r0 + threadIdx.x;
    if (d < D) {
      const C* r = n + d * KS;
      int64_t nd = 0;
      for (int k = 0; k < K; ++k) nd += r[k];
      den[threadIdx.x] = (float)nd + den_add;
    }
    __syncthreads();
    const int64_t rows = D - r0 < 256 ? D - r0 : 256;
    const int64_t cells = rows * KS;
    const C* src = n + r0 * KS;
    float* dst = th + r0 * KS;
    for (int64_t i = threadIdx.x; i < cells; i += 256) {
      const int k = (int)(i % KS);
      dst[i] = k < K ? ((float)src[i] + add) / den[i / KS] : 0.f;
    }
    __syncthreads();
  }
}

template <typename C, typename CK>
__global__ __launch_bounds__(256) void k_phi_rows(const C* __restrict__ nw, const CK* __restrict__ nk,
                                                  int64_t V, int K, int KS, float add, float vb,
                                                  float* __restrict__ ph) {
  __shared__ float den[256];
  for (int k = threadIdx.x; k < KS; k += blockDim.x) den[k] = (float)nk[k] + vb;
  __syncthreads();
  const int64_t n = V * KS;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int k = (int)(i % KS);
    ph[i] = k < K ? ((float)nw[i] + add) / den[k] : 0.f;
  }
}

}  // namespace

// part: scratch of [grid][8] doubles (grid = oni_tail_grid()); out: [8] doubles
ONI_API int oni_tail_grid() { return 512; }

ONI_API int oni_tail_sums(const int32_t* nwk, const float* q, const int32_t* nk, const int32_t* ndk, int64_t V,
                          int64_t D, int K, int KS, double alpha, double beta, double vbeta, double kalpha,
                          double* part, double* out, hipStream_t s) {
  if (K < 1 || K > KS || KS > 256) return (int)hipErrorInvalidValue;
  const int grid = 512;
  k_tail_partials<<<grid, kTailBlock, 0, s>>>(nwk, q, nk, ndk, V, D, K, KS, alpha, beta, vbeta, kalpha, part);
  k_tail_final<<<1, kTailVals * 64, 0, s>>>(part, grid, out);
  return (int)hipGetLastError();
}

// csize: bytes per count (4: int32 tables, 8: int64 posterior-average sums)
ONI_API int oni_theta_rows(const void* n, int64_t D, int K, int KS, float add, float den_add, float* th, int csize,
                           hipStream_t s) {
  if (K < 1 || K > KS || (csize != 4 && csize != 8)) return (int)hipErrorInvalidValue;
  if (D <= 0) return 0;
  const unsigned grid = oni::grid_for(D, 256, 2048);
  if (csize == 8)
    k_theta_rows<int64_t><<<grid, 256, 0, s>>>(static_cast<const int64_t*>(n), D, K, KS, add, den_add, th);
  else
    k_theta_rows<int32_t><<<grid, 256, 0, s>>>(static_cast<const int32_t*>(n), D, K, KS, add, den_add, th);
  return (int)hipGetLastError();
}

// csize / ksize: bytes per count of nw / nk (4 or 8)
ONI_API int oni_phi_rows(const void* nw, const void* nk, int64_t V, int K, int KS, float add, float vb, float* ph,
                         int csize, int ksize, hipStream_t s) {
  if (K < 1 || K > KS || KS > 256 || (csize != 4 && csize != 8) || (ksize != 4 && ksize != 8))
    return (int)hipErrorInvalidValue;
  if (V <= 0) return 0;
  const unsigned grid = oni::grid_for(V * KS, 256, 4096);
#define ONI_PHI(C, CK)                                                                                      \
  k_phi_rows<C, CK><<<grid, 256, 0, s>>>(static_cast<const C*>(nw), static_cast<const CK*>(nk), V, K, KS, add, \
                                         vb, ph)
  if (csize == 8 && ksize == 8) ONI_PHI(int64_t, int64_t);
  else if (csize == 8) ONI_PHI(int64_t, int32_t);
  else if (ksize == 8) ONI_PHI(int32_t, int64_t);
  else ONI_PHI(int32_t, int32_t);
#undef ONI_PHI
  return (int)hipGetLastError();
}
