// K10/K11/K12 -- collapsed-Gibbs LDA on CDNA4: init, sweep, delta-apply (+ q-table refresh).
//
// Replaces oni-lda-c's variational-EM `lda est` E-step/M-step loop (lda-estimate.c run_em /
// doc_e_step, lda-inference.c, lda-model.c lda_mle; SURVEY.md §3.2, [U-H]) with collapsed Gibbs
// sampling, as the north star requires (BASELINE.json).
//
// Execution model (MI355X-first, not a translation of anything):
//  * Documents (IPs) are owned by sampler "units" of G lanes. A unit walks one chunk (≤ L tokens
//    of one doc) sequentially, holding the doc's topic counts n_dk IN REGISTERS (KP per lane,
//    KS = G*KP padded topics), so the doc side is exact Gibbs within a chunk.
//  * The word side samples against the sweep-start table q[w,k] = (n_wk+β)/(n_k+Vβ)
//    (AD-LDA staleness, one snapshot per sweep). Topic moves are accumulated as int32 deltas
//    (dnwk, dnk); in data-parallel runs that buffer is what RCCL all-reduces over xGMI.
//  * A wave = one SELL slice of S = 64/G chunks; tokens are step-major so per-step word/topic
//    loads are coalesced. The q row is re-used while consecutive tokens share a word (tokens of
//    one (doc, word) pair are adjacent).
//  * G = 1 for K ≤ 32 (one lane owns all topics: no cross-lane traffic at all); G ∈ {2, 4, 8, 16}
//    above (2 lanes up to K = 56, 4 up to 112) with DPP / __shfl_up scans across the unit.
//  * Draws are Philox4x32-10 keyed by (seed) with counter (pos/4, doc key, sweep, stream): the
//    chain is a pure function of the data + seed — bitwise identical for any GPU count, shard
//    plan, chunk packing or resume point (tested against the NumPy oracle, oni355/ref/spec.py).
//  * Long documents span several chunks. Those chunks start from the sweep-start row of ndk_src
//    and add their deltas into ndk_dst (pre-copied row), with integer atomics: still order-free.
#include "gibbs_sampler.h"

namespace {

// Posterior-average sums += four int32 counts at vector i: int64 sums where S samples of the
// table's largest count could pass 2^31 (the host decides per table), else int32 (half the bytes).
__device__ __forceinline__ void add_counts(void* __restrict__ base, int64_t i, const int4 v, int wide) {
  if (wide) {
    longlong2* q = reinterpret_cast<longlong2*>(static_cast<int64_t*>(base) + i * 4);
    longlong2 a = q[0], b = q[1];
    a.x += v.x; a.y += v.y; b.x += v.z; b.y += v.w;
    q[0] = a;
    q[1] = b;
  } else {
    int4* q = static_cast<int4*>(base) + i;
    int4 a = *q;
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    *q = a;
  }
}

// Delta apply + q refresh: n_wk += Δ; n_k' = n_k + Δn_k; q = (n_wk+β)/(n_k'+Vβ); the token-exclusion
// constants qfix = (A, B) with D = n_k' + Vβ, A = D/(D−1), B = 1/(D−1) (A = 1, B = 0 for empty
// topics; see gibbs_sampler.h); zero the other delta buffer for the next sweep; bump the device
// sweep counter. nk/dnwk are ping-ponged by the
// host so no block ever reads what another block of this launch writes.
// With n_rows > 0 the same launch also seeds the NEXT sweep's long-document rows (rdst[r] :=
// rsrc[r]: chunked documents add their Δn_dk atomically into a copy of the current counts), which
// saves the separate k_copy_rows launch per sweep.
__global__ __launch_bounds__(256) void k_apply(int32_t* __restrict__ nwk, const int32_t* __restrict__ dcur,
                                                int32_t* __restrict__ dother, const int32_t* __restrict__ nk_cur,
                                                int32_t* __restrict__ nk_next, float* __restrict__ q,
                                                float* __restrict__ qfix, int64_t V,
                                                int K, int KS, float beta, float vbeta, uint32_t* sweep_ctr,
                                                int bump, int absolute, int nk_rep, const int32_t* __restrict__ rsrc,
                                                int32_t* __restrict__ rdst, const int32_t* __restrict__ rows,
                                                int64_t n_rows, void* __restrict__ acc_wk, void* __restrict__ acc_k,
                                                void* __restrict__ acc_dk, int acc_wide,
                                                const int32_t* __restrict__ ndk_fin, int64_t D, int inplace) {
  __shared__ float den[256];
  __shared__ int32_t nkn[256];
  __shared__ int32_t part[256];
  const int32_t* dnk_cur = dcur + V * KS;
  // Σ over the nk_rep Δn_k replicas, spread over the whole block (256/KS replica groups, ≤ 3
  // loads per thread at K = 20) instead of one serial 32-load chain per topic: integer sums, so
  // the result is order-independent
  {
    const int groups = (int)blockDim.x / KS;
    const int k = (int)threadIdx.x % KS, gi = (int)threadIdx.x / KS;
    int32_t v = 0;
    if (gi < groups)
      for (int r = gi; r < nk_rep; r += groups) v += dnk_cur[r * KS + k];
    part[threadIdx.x] = v;
    __syncthreads();
    if ((int)threadIdx.x < KS) {
      int32_t t = nk_cur[threadIdx.x];
      for (int g2 = 0; g2 < groups; ++g2) t += part[g2 * KS + threadIdx.x];
      nkn[threadIdx.x] = t;
      den[threadIdx.x] = (float)t + vbeta;
    }
  }
  __syncthreads();
  if (blockIdx.x == 0) {
    for (int k = threadIdx.x; k < KS; k += blockDim.x) {
      nk_next[k] = nkn[k];
      const float dm1 = den[k] - 1.0f;
      const bool ok = k < K && nkn[k] >= 1;
      qfix[k] = ok ? den[k] / dm1 : 1.0f;
      qfix[KS + k] = ok ? 1.0f / dm1 : 0.0f;
    }
    for (int k = threadIdx.x; k < nk_rep * KS + kDnAux; k += blockDim.x) dother[V * KS + k] = 0;
    if (threadIdx.x == 0 && bump) *sweep_ctr += 1u;
    if (acc_k)
      for (int k = threadIdx.x; k < KS; k += blockDim.x) {
        if (acc_wide & 2) static_cast<int64_t*>(acc_k)[k] += nkn[k];
        else static_cast<int32_t*>(acc_k)[k] += nkn[k];
      }
  }
  const int64_t nvec = V * KS / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    int4 nv;
    if (inplace) {
      // the count pass already added this sweep's Δn_wk into n_wk (one process, no X01): the Δ
      // heads are never written, so neither read nor zeroed -- 2 of the 5 table passes
      nv = reinterpret_cast<const int4*>(nwk)[i];
    } else {
      const int4 dv = reinterpret_cast<const int4*>(dcur)[i];
      nv = dv;
      if (!absolute) {
        nv = reinterpret_cast<int4*>(nwk)[i];
        nv.x += dv.x; nv.y += dv.y; nv.z += dv.z; nv.w += dv.w;
      }
      reinterpret_cast<int4*>(nwk)[i] = nv;
      reinterpret_cast<int4*>(dother)[i] = make_int4(0, 0, 0, 0);
    }
    if (acc_wk) add_counts(acc_wk, i, nv, acc_wide & 1);
    const int k0 = (int)((i * 4) % KS);
    float4 qo;
    qo.x = k0 + 0 < K ? ((float)nv.x + beta) / den[k0 + 0] : 0.f;
    qo.y = k0 + 1 < K ? ((float)nv.y + beta) / den[k0 + 1] : 0.f;
    qo.z = k0 + 2 < K ? ((float)nv.z + beta) / den[k0 + 2] : 0.f;
    qo.w = k0 + 3 < K ? ((float)nv.w + beta) / den[k0 + 3] : 0.f;
    reinterpret_cast<float4*>(q)[i] = qo;
  }
  const int64_t rtotal = n_rows * KS;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rtotal; i += stride) {
    const int64_t r = rows[i / KS];
    const int k = (int)(i % KS);
    rdst[r * KS + k] = rsrc[r * KS + k];
  }
  if (acc_dk) {
    const int64_t dvec = D * KS / 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < dvec; i += stride)
      add_counts(acc_dk, i, reinterpret_cast<const int4*>(ndk_fin)[i], acc_wide & 4);
  }
}

// Exactness guard of the row-f32 samplers (k_gibbs_x1 / k_gibbs_ldsg keep n + α as f32 in their
// rows): *flag := 1 iff every count of the given rows (the documents long enough to matter) is at
// most `limit` -- the largest sweep-start count whose chunk can still move it by L without leaving
// the exactly representable range. One block, before the sweep's sampler (inside its graph).
__global__ __launch_bounds__(256) void k_exact_guard(const int32_t* __restrict__ ndk, const int32_t* __restrict__ rows,
                                                     int64_t n_rows, int KS, int K, int32_t limit,
                                                     int32_t* __restrict__ flag) {
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  int b = 0;
  for (int64_t i = threadIdx.x; i < n_rows * K; i += blockDim.x) {
    const int64_t r = rows[i / K];
    b |= ndk[r * KS + (int)(i % K)] > limit;
  }
  if (b) atomicOr(&bad, 1);
  __syncthreads();
  if (threadIdx.x == 0) *flag = bad ? 0 : 1;
}

__global__ void k_copy_rows(const int32_t* __restrict__ src, int32_t* __restrict__ dst,
                            const int32_t* __restrict__ rows, int64_t n_rows, int KS) {
  const int64_t total = n_rows * KS;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t r = rows[i / KS];
    const int k = (int)(i % KS);
    dst[r * KS + k] = src[r * KS + k];
  }
}

// Delta recount (MODE 2): only tokens whose topic changed this sweep (per-step ballot masks,
// an L2-resident bitmap: 1 bit per SELL slot) touch the z arrays. Tokens are visited in
// word-sorted order; a changed token adds -1 at (w, z_prev) and +1 at (w, z) to the block's LDS
// table and refreshes z_prev; non-zero cells are flushed as row-contiguous atomics into Δn_wk.
// The word id of a changed token is re-read from the SELL word array (only ~5% of tokens), so
// the per-token stream is the 4-byte slot index alone.
__global__ __launch_bounds__(256) void k_delta_recount(const int32_t* __restrict__ wslot,
                                                        const int32_t* __restrict__ tile_wlo,
                                                        const int32_t* __restrict__ tile_whi,
                                                        const uint64_t* __restrict__ mask,
                                                        const uint32_t* __restrict__ tok_word,
                                                        const uint8_t* __restrict__ tok_z,
                                                        uint8_t* __restrict__ tok_zprev, int64_t T,
                                                        int32_t* __restrict__ dnwk, int KS, int log2S, int G,
                                                        int tile, int wmax) {
  extern __shared__ __attribute__((aligned(16))) int32_t hst[];
  const int64_t lo = (int64_t)blockIdx.x * tile;
  if (lo >= T) return;
  const int64_t hi = lo + tile < T ? lo + tile : T;
  const int w_lo = tile_wlo[blockIdx.x], w_hi = tile_whi[blockIdx.x];
  const int rows = (w_hi - w_lo + 1) < wmax ? (w_hi - w_lo + 1) : wmax;
  const int cells = rows * KS;
  for (int i = threadIdx.x; i < cells; i += blockDim.x) hst[i] = 0;
  __syncthreads();
  const int64_t Smask = (1ll << log2S) - 1;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const int64_t slot = __builtin_nontemporal_load(&wslot[i]);
    const uint64_t m = mask[slot >> log2S];
    const int bit = (int)(slot & Smask) * G;
    if ((m >> bit) & 1ull) {
      const int w = (int)tok_word[slot];
      const int zn = tok_z[slot];
      const int zo = tok_zprev[slot];
      tok_zprev[slot] = (uint8_t)zn;
      const int r = w - w_lo;
      if (r < rows) {
        atomicAdd(&hst[r * KS + zn], 1);
        atomicAdd(&hst[r * KS + zo], -1);
      } else {
        atomicAdd(&dnwk[(int64_t)w * KS + zn], 1);
        atomicAdd(&dnwk[(int64_t)w * KS + zo], -1);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < cells; i += blockDim.x) {
    const int v = hst[i];
    if (v) atomicAdd(&dnwk[(int64_t)(w_lo + i / KS) * KS + (i % KS)], v);
  }
}

// K11 (option B of SURVEY.md §7.4.3): rebuild the local n_wk table from z with NO global
// per-token atomics. Tokens are visited in word-sorted order (wsorted/wslot built once with the
// corpus); each block owns a contiguous run of them, histograms (word, topic) in LDS (rows = the
// block's word span, capped at wmax; the tail of a very wide span goes straight to global), and
// flushes one row-contiguous atomic per non-zero (word, topic) cell. The topic gather z[wslot]
// reads 1 byte per token from the (L2/MALL-resident) SELL topic array.
// Word-sorted recount tile: 4096 tokens, 256 threads × 16 CONTIGUOUS tokens each, loaded with
// 16-B vector loads up front (one memory round trip per thread instead of a dependent
// load→atomic chain per token), counted into an LDS histogram of the tile's word rows, flushed
// with one global atomic per non-zero cell. The LDS histogram is capped at kRecountCells cells
// (8 KB) so ≥ 8 blocks fit per CU — a 64 KB cap left 2 waves per SIMD and made the kernel
// latency-bound; rows beyond the cap (tail tiles of rare words) go straight to global atomics.
constexpr int kRecountTile = 4096;
constexpr int kRecountCells = 2048;

// E tokens per lane: 16 (4096-token tiles) for large corpora; 4 (1024-token tiles) below 8M
// tokens, where 4096-token tiles leave fewer workgroups than the chip holds (a 2M-token DNS day:
// 488 of them on 256 CUs)
template <int E>
__global__ __launch_bounds__(256) void k_recount(const int32_t* __restrict__ wsorted, const int32_t* __restrict__ wslot,
                                                  const uint8_t* __restrict__ tok_z, int64_t T, int32_t* __restrict__ nwk,
                                                  int KS) {
  static_assert(E % 4 == 0, "whole 16-B loads");
  constexpr int kTile = 256 * E;
  __shared__ int32_t hst[kRecountCells];
  const int64_t lo = (int64_t)blockIdx.x * kTile;
  if (lo >= T) return;
  const int64_t hi = lo + kTile < T ? lo + kTile : T;
  const int w_lo = wsorted[lo], w_hi = wsorted[hi - 1];
  const int cap_rows = kRecountCells / KS;
  const int rows = (w_hi - w_lo + 1) < cap_rows ? (w_hi - w_lo + 1) : cap_rows;
  const int cells = rows * KS;
  for (int i = threadIdx.x; i < cells; i += blockDim.x) hst[i] = 0;
  const int64_t base = lo + (int64_t)threadIdx.x * E;
  int w[E], z[E];
  int nt = 0;
  if (base + E <= hi) {
    nt = E;
    const int4* wp = reinterpret_cast<const int4*>(wsorted + base);
#pragma unroll
    for (int q = 0; q < E / 4; ++q) {
      const int4 v = wp[q];
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
    if (wslot) {
      const int4* sp = reinterpret_cast<const int4*>(wslot + base);
      int sl[E];
#pragma unroll
      for (int q = 0; q < E / 4; ++q) {
        const int4 v = sp[q];
        sl[4 * q] = v.x; sl[4 * q + 1] = v.y; sl[4 * q + 2] = v.z; sl[4 * q + 3] = v.w;
      }
#pragma unroll
      for (int t = 0; t < E; ++t) z[t] = tok_z[sl[t]];
    } else {
#pragma unroll
      for (int q = 0; q < E / 4; ++q) {
        const uint32_t zz = *reinterpret_cast<const uint32_t*>(tok_z + base + 4 * q);
#pragma unroll
        for (int t = 0; t < 4; ++t) z[4 * q + t] = (int)((zz >> (8 * t)) & 0xFFu);
      }
    }
  } else if (base < hi) {
    nt = (int)(hi - base);
    for (int t = 0; t < nt; ++t) {
      w[t] = wsorted[base + t];
      z[t] = wslot ? tok_z[wslot[base + t]] : tok_z[base + t];
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < E; ++t) {
    if (t < nt) {
      const int r = w[t] - w_lo;
      if (r < rows) atomicAdd(&hst[r * KS + z[t]], 1);
      else atomicAdd(&nwk[(int64_t)w[t] * KS + z[t]], 1);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < cells; i += blockDim.x) {
    const int v = hst[i];
    if (v) atomicAdd(&nwk[(int64_t)(w_lo + i / KS) * KS + (i % KS)], v);
  }
}

// Streaming recount for KS ≤ 32 (dual-z mode): z_w is word-sorted, so each thread takes 16
// CONTIGUOUS tokens (one 64-B word-id load + one 16-B topic load), counts them in a register
// histogram while the word stays the same (frequent words dominate by tokens), and only flushes
// non-zero bins to the block's LDS table when the word changes. This removes the LDS-atomic
// hot spots of one-atomic-per-token (tokens of a frequent word share a handful of topics).
template <int KS>
__global__ __launch_bounds__(256) void k_recount_reg(const int32_t* __restrict__ wsorted, const uint8_t* __restrict__ z_w,
                                                      int64_t T, int32_t* __restrict__ nwk, int tile, int wmax) {
  extern __shared__ __attribute__((aligned(16))) int32_t hst[];
  constexpr int E = 16;
  const int64_t lo = (int64_t)blockIdx.x * tile;
  if (lo >= T) return;
  const int64_t hi = lo + tile < T ? lo + tile : T;
  const int w_lo = wsorted[lo], w_hi = wsorted[hi - 1];
  const int rows = (w_hi - w_lo + 1) < wmax ? (w_hi - w_lo + 1) : wmax;
  const int cells = rows * KS;
  for (int i = threadIdx.x; i < cells; i += blockDim.x) hst[i] = 0;
  __syncthreads();
  int cnt[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) cnt[k] = 0;
  int cur = -1;
  auto flush = [&](int w) {
    if (w < 0) return;
    const int r = w - w_lo;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      if (cnt[k]) {
        if (r < rows) atomicAdd(&hst[r * KS + k], cnt[k]);
        else atomicAdd(&nwk[(int64_t)w * KS + k], cnt[k]);
        cnt[k] = 0;
      }
    }
  };
  for (int64_t t0 = lo + (int64_t)threadIdx.x * E; t0 < hi; t0 += (int64_t)blockDim.x * E) {
    int wv[E];
    uint8_t zv[E];
    const int n = (int)(hi - t0 < E ? hi - t0 : E);
    if (n == E) {
#pragma unroll
      for (int q = 0; q < E; q += 4) {
        const int4 v = *reinterpret_cast<const int4*>(wsorted + t0 + q);
        wv[q] = v.x; wv[q + 1] = v.y; wv[q + 2] = v.z; wv[q + 3] = v.w;
      }
      const uint4 zz = *reinterpret_cast<const uint4*>(z_w + t0);
      const uint32_t zw[4] = {zz.x, zz.y, zz.z, zz.w};
#pragma unroll
      for (int q = 0; q < E; ++q) zv[q] = (uint8_t)(zw[q >> 2] >> (8 * (q & 3)));
    } else {
#pragma unroll
      for (int q = 0; q < E; ++q) {
        wv[q] = q < n ? wsorted[t0 + q] : -1;
        zv[q] = q < n ? z_w[t0 + q] : 0;
      }
    }
#pragma unroll
    for (int q = 0; q < E; ++q) {
      if (q >= n) break;
      if (wv[q] != cur) {
        flush(cur);
        cur = wv[q];
      }
#pragma unroll
      for (int k = 0; k < KS; ++k) cnt[k] += (k == (int)zv[q]);
    }
  }
  flush(cur);
  __syncthreads();
  for (int i = threadIdx.x; i < cells; i += blockDim.x) {
    const int v = hst[i];
    if (v) atomicAdd(&nwk[(int64_t)(w_lo + i / KS) * KS + (i % KS)], v);
  }
}

// Word-bitmap delta recount (MODE 4). A block owns 256 bitmap words = 8192 word-sorted token
// positions; each thread reads one 32-bit word (coalesced 1 KB per block), clears it, and for
// each set bit reads the position's packed record zz_w = (old | new << 8) | row << 16, row = its
// word minus the block's first word (written once with the corpus; 0xFFFF = too far, read
// wsorted) -- one contiguous 4-B array in word-sorted order, touched only where a token changed.
// At 5-10 % changed tokens nearly every 128-B line of it is touched, so the record carrying the
// row (instead of a second 4-B wsorted gather) is a third less traffic per sweep. Deltas go to
// an LDS table over the block's word span (rows capped at wmax; wider spans go straight to
// global atomics) and are flushed one row-contiguous atomic per non-zero cell. Cost ∝ changed
// tokens + T/8 bytes of bitmap, vs the slot-indexed delta recount's 4 B/token scan.
constexpr int kWBitsPerBlock = 256 * 32;

__global__ __launch_bounds__(256) void k_wdelta_recount(uint32_t* __restrict__ wbits,
                                                         const int32_t* __restrict__ wsorted,
                                                         const uint32_t* __restrict__ zz_w, int64_t T,
                                                         int32_t* __restrict__ dnwk, int KS, int wmax) {
  extern __shared__ __attribute__((aligned(16))) int32_t hst[];
  const int64_t lo = (int64_t)blockIdx.x * kWBitsPerBlock;
  if (lo >= T) return;
  const int64_t hi = lo + kWBitsPerBlock < T ? lo + kWBitsPerBlock : T;
  const int w_lo = wsorted[lo], w_hi = wsorted[hi - 1];
  const int rows = (w_hi - w_lo + 1) < wmax ? (w_hi - w_lo + 1) : wmax;
  const int cells = rows * KS;
  for (int i = threadIdx.x; i < cells; i += blockDim.x) hst[i] = 0;
  __syncthreads();
  const int64_t word = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t m = 0;
  if (word * 32 < T) {
    m = wbits[word];
    if (m) wbits[word] = 0u;
  }
  // four set bits per round: their record loads are issued together (one latency, not four)
  while (m) {
    uint32_t zz[4];
    int64_t pos[4];
    bool v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = m != 0u;
      const int b = v[j] ? __ffs(m) - 1 : 0;
      m &= v[j] ? m - 1u : m;
      pos[j] = word * 32 + b;
      zz[j] = zz_w[pos[j]];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!v[j]) continue;
      const int zo = (int)(zz[j] & 0xFFu), zn = (int)((zz[j] >> 8) & 0xFFu);
      int r = (int)(zz[j] >> 16);
      if (r == 0xFFFF) r = wsorted[pos[j]] - w_lo;
      if (r < rows) {
        atomicAdd(&hst[r * KS + zn], 1);
        atomicAdd(&hst[r * KS + zo], -1);
      } else {
        const int64_t w = (int64_t)w_lo + r;
        atomicAdd(&dnwk[w * KS + zn], 1);
        atomicAdd(&dnwk[w * KS + zo], -1);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < cells; i += blockDim.x) {
    const int v = hst[i];
    if (v) atomicAdd(&dnwk[(int64_t)(w_lo + i / KS) * KS + (i % KS)], v);
  }
}

}  // namespace

ONI_API int oni_wdelta_recount(uint32_t* wbits, const int32_t* wsorted, const uint32_t* zz_w, int64_t T,
                               int32_t* dnwk, int KS, int wmax, hipStream_t s) {
  if (T == 0) return 0;
  if (wmax < 1 || KS < 1 || (size_t)wmax * KS * 4 > 64 * 1024) return (int)hipErrorInvalidValue;
  const unsigned grid = (unsigned)((T + kWBitsPerBlock - 1) / kWBitsPerBlock);
  k_wdelta_recount<<<grid, 256, (size_t)wmax * KS * 4, s>>>(wbits, wsorted, zz_w, T, dnwk, KS, wmax);
  return (int)hipGetLastError();
}

ONI_API int oni_recount_stream(const int32_t* wsorted, const uint8_t* z_w, int64_t T, int32_t* nwk, int KS, int tile,
                               int wmax, hipStream_t s) {
  if (T == 0) return 0;
  if (tile % (256 * 16) != 0 || wmax < 1 || (size_t)wmax * KS * 4 > 64 * 1024) return (int)hipErrorInvalidValue;
  const unsigned grid = (unsigned)((T + tile - 1) / tile);
  const size_t lds = (size_t)wmax * KS * 4;
#define ONI_RC(ks_)                                                                       \
  if (KS == ks_) {                                                                        \
    k_recount_reg<ks_><<<grid, 256, lds, s>>>(wsorted, z_w, T, nwk, tile, wmax);          \
    return (int)hipGetLastError();                                                        \
  }
  ONI_RC(4) ONI_RC(8) ONI_RC(12) ONI_RC(16) ONI_RC(20) ONI_RC(24) ONI_RC(28) ONI_RC(32)
#undef ONI_RC
  return (int)hipErrorInvalidValue;
}

// Supported (G, KP) configurations. K ≤ 32: G = 1 (KP = K rounded up to 4).
ONI_API int oni_gibbs_launch(const OniGibbs* a, int G, int KP, int init, int mode, int qpf, hipStream_t s) {
  if (a->nk_rep < 1 || (a->nk_rep & (a->nk_rep - 1))) return (int)hipErrorInvalidValue;
  if (a->K < 1 || a->K > 255 || a->K > a->KS || mode < 0 || mode > 4) return (int)hipErrorInvalidValue;
  if (mode == 2 && !a->chg_mask) return (int)hipErrorInvalidValue;
  if (mode == 3 && (!a->wpos || !a->z_w)) return (int)hipErrorInvalidValue;
  if (mode == 4 && (!a->wpos || !a->zz_w || !a->chg_mask)) return (int)hipErrorInvalidValue;
  switch (G) {
    case 1: return oni_gibbs_dispatch_g1(*a, KP, init != 0, mode, qpf, s);
    case 2: return oni_gibbs_dispatch_g2(*a, KP, init != 0, mode, qpf, s);
    case 4: return oni_gibbs_dispatch_g4(*a, KP, init != 0, mode, qpf, s);
    case 8:
    case 16: return oni_gibbs_dispatch_g8(*a, G, KP, init != 0, mode, qpf, s);
    default: break;
  }
  return (int)hipErrorInvalidValue;
}

ONI_API int oni_gibbs_sizeof_args() { return (int)sizeof(OniGibbs); }

ONI_API int oni_exact_guard(const int32_t* ndk, const int32_t* rows, int64_t n_rows, int KS, int K, int32_t limit,
                            int32_t* flag, hipStream_t s) {
  if (n_rows < 0 || K < 1 || K > KS || flag == nullptr) return (int)hipErrorInvalidValue;
  k_exact_guard<<<1, 256, 0, s>>>(ndk, rows, n_rows, KS, K, limit, flag);
  return (int)hipGetLastError();
}

// rsrc/rdst/rows/n_rows: optional fused long-row copy for the next sweep (n_rows = 0: none).
// inplace: Δn_wk was added straight into nwk by the count pass (world 1); only q, n_k, the Δn_k
// replicas and the aux words are handled here.
// acc_wk/acc_k/acc_dk (all or none): the posterior-average sums ([V, KS], [KS], [D, KS]; int64 where
// bit 0 / 1 / 2 of acc_wide is set, else int32) gain this sweep's n_wk, n_k and doc rows ndk_fin
// [D, KS] -- the sample add in the same pass.
ONI_API int oni_gibbs_apply(int32_t* nwk, const int32_t* dcur, int32_t* dother, const int32_t* nk_cur,
                            int32_t* nk_next, float* q, float* qfix, int64_t V, int K, int KS, float beta, float vbeta,
                            uint32_t* sweep_ctr, int bump, int absolute, int nk_rep, const int32_t* rsrc,
                            int32_t* rdst, const int32_t* rows, int64_t n_rows, void* acc_wk, void* acc_k,
                            void* acc_dk, int acc_wide, const int32_t* ndk_fin, int64_t D, int inplace,
                            hipStream_t s) {
  if (inplace && absolute) return (int)hipErrorInvalidValue;
  if (KS % 4 != 0 || KS > 256 || nk_rep < 1 || (nk_rep & (nk_rep - 1)) || qfix == nullptr)
    return (int)hipErrorInvalidValue;
  if (n_rows < 0 || (n_rows > 0 && (rsrc == nullptr || rdst == nullptr || rows == nullptr)))
    return (int)hipErrorInvalidValue;
  const bool acc = acc_wk != nullptr;
  if (acc != (acc_k != nullptr) || acc != (acc_dk != nullptr) || (acc && (ndk_fin == nullptr || D < 0)))
    return (int)hipErrorInvalidValue;
  int64_t work = V * KS / 4 > n_rows * KS ? V * KS / 4 : n_rows * KS;
  if (acc && D * KS / 4 > work) work = D * KS / 4;
  k_apply<<<oni::grid_for(work, 256, 2048), 256, 0, s>>>(nwk, dcur, dother, nk_cur, nk_next, q, qfix, V, K, KS, beta,
                                                          vbeta, sweep_ctr, bump, absolute, nk_rep, rsrc, rdst, rows,
                                                          n_rows, acc_wk, acc_k, acc ? acc_dk : nullptr, acc_wide,
                                                          ndk_fin, acc ? D : 0, inplace);
  return (int)hipGetLastError();
}

ONI_API int oni_recount(const int32_t* wsorted, const int32_t* wslot, const uint8_t* tok_z, int64_t T, int32_t* nwk,
                        int KS, int tile, int wmax, hipStream_t s) {
  if (T == 0) return 0;
  if (KS < 1 || KS > kRecountCells) return (int)hipErrorInvalidValue;
  (void)tile;
  (void)wmax;
  if (T < (int64_t(8) << 20)) {
    const unsigned grid = (unsigned)((T + 1023) / 1024);
    k_recount<4><<<grid, 256, 0, s>>>(wsorted, wslot, tok_z, T, nwk, KS);
  } else {
    const unsigned grid = (unsigned)((T + kRecountTile - 1) / kRecountTile);
    k_recount<16><<<grid, 256, 0, s>>>(wsorted, wslot, tok_z, T, nwk, KS);
  }
  return (int)hipGetLastError();
}

ONI_API int oni_delta_recount(const int32_t* wslot, const int32_t* tile_wlo, const int32_t* tile_whi,
                              const uint64_t* mask, const uint32_t* tok_word, const uint8_t* tok_z, uint8_t* tok_zprev,
                              int64_t T, int32_t* dnwk, int KS, int log2S, int G, int tile, int wmax, hipStream_t s) {
  if (T == 0) return 0;
  if (tile < 256 || wmax < 1 || (size_t)wmax * KS * 4 > 64 * 1024) return (int)hipErrorInvalidValue;
  const unsigned grid = (unsigned)((T + tile - 1) / tile);
  k_delta_recount<<<grid, 256, (size_t)wmax * KS * 4, s>>>(wslot, tile_wlo, tile_whi, mask, tok_word, tok_z, tok_zprev,
                                                            T, dnwk, KS, log2S, G, tile, wmax);
  return (int)hipGetLastError();
}

ONI_API int oni_copy_rows(const int32_t* src, int32_t* dst, const int32_t* rows, int64_t n_rows, int KS,
                          hipStream_t s) {
  if (n_rows == 0) return 0;
  k_copy_rows<<<oni::grid_for(n_rows * KS), 256, 0, s>>>(src, dst, rows, n_rows, KS);
  return (int)hipGetLastError();
}
