// K10 variant "ws": word-sparse collapsed-Gibbs sweep for large K.
//
// The dense samplers spend K multiply-adds per token on p_k = (n_dk + α)·q_wk. Split the word
// factor q_wk = (n_wk + β)/(n_k + Vβ) = a_wk + b_k with a_wk = n_wk/(n_k + Vβ) and b_k =
// β/(n_k + Vβ):
//
//     p_k = (n_dk + α)·a_wk   [word bucket: only the topics the word holds, n_wk > 0]
//         + (n_dk + α)·b_k    [smoothing bucket: every topic, total R_d]
//
// (SparseLDA's word and smoothing buckets). What makes them cheap on this machine is the AD-LDA
// sweep: the word side is a sweep-start snapshot, so every word's non-zero-topic list
// (k ascending, a_wk) and the b table are STATIC for the whole sweep -- built once per sweep by
// k_ws_tables right after the q refresh, no sparse structure is maintained while sampling. A
// token then costs |list(w)| fma instead of K (flow day at K = 100: 6.9 topics per word
// token-weighted, 21 at a wave step's slowest lane, against 112 padded; profiles/r3/
// k100_count_sparsity.jsonl); R_d is kept per chain with one subtract and one add per token.
//
// Execution model: one lane per chunk, one wave per block (64 chunks: one SELL slice of a G = 1
// corpus, or G consecutive slices of a corpus laid out for the dense G-lane samplers). The chunk's doc counts live in LDS, topic-major ([k][lane]: lanes reading the same
// topic hit distinct banks), because the word bucket reads them at data-dependent topics --
// registers can only be indexed statically. The current word's list sits in registers (up to
// kWsE entries, refetched on a word change); longer lists continue from the table (slow path,
// common only in the first sweeps, which the model runs on the dense sampler).
//
// Numerics (replayed bit for bit by oni355/ref/spec.py gibbs_pass_ws):
//   chunk start  R = fma chain over k = 0..K-1 of (n_k + α)·b_k
//   per token    n_zo -= 1; R = R - b_zo
//                W_j = fma(n_kj + α, a_j, W_{j-1}) over the word's list (W_-1 = 0); W = W_last
//                thr = u01(r) · (W + R)
//                thr < W:  z = k_j for the first j with W_j > thr
//                otherwise t = thr - W; z = first k with fma chain of (n_k + α)·b_k > t (K-1 if none)
//                n_z += 1; R = R + b_z
// Same Philox draw per token as every other sampler (position, doc key, sweep, stream 1).
#include <type_traits>

#include "gibbs_sampler.h"

struct OniWsTabs {
  const int32_t* llen;  // [V] number of topics with n_wk > 0 (k < K)
  const uint8_t* lk;    // [V][KS] those topics, ascending
  const float* la;      // [V][KS] a_wk = n_wk / (n_k + Vβ), same order
  const float* b;       // [KS] b_k = β / (n_k + Vβ); 0 for k ≥ K
  unsigned long long* stats;  // optional [5]: tokens, smoothing-bucket draws, slow-path lists, Σ wave-step list max, wave steps
  const uint32_t* lofs;       // [V] for G-lane units (k_gibbs_wsg): byte g = first list entry of lane g's topics
};

namespace {

constexpr int kWsE = 32;  // register capacity of the current word's topic list

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int m = 1; m < oni::kWave; m <<= 1) v += __shfl_xor(v, m);
  return v;
}

template <int MODE, bool AIR>
__global__ __launch_bounds__(64) void k_gibbs_ws(const OniGibbs a, const OniWsTabs t, int KR, int G) {
  extern __shared__ float ws_lds[];
  const int lane = threadIdx.x;
  const int K = a.K, KS = a.KS;
  // the corpus may be laid out for G-lane units (S = 64/G chunks per slice, shared with the dense
  // samplers): the wave then takes G consecutive slices, one lane per chunk. Slices are sorted
  // by length, so the first one bounds the wave's steps.
  const int S = oni::kWave / G;
  const int sq = lane / S, c = lane % S;
  float* row = ws_lds;                                            // [KR][64] n_dk (+ α)
  float* bt = ws_lds + (size_t)KR * 64;                           // [KR] b_k
  int32_t* cdoc = reinterpret_cast<int32_t*>(bt + KR);            // [64] chunk docs
  int32_t* cmul = cdoc + 64;                                      // [64] chunk multi flags
  const int64_t slice0 = (int64_t)blockIdx.x * G;
  const int64_t slice = slice0 + sq;
  const bool valid = slice < a.n_slices;
  const int64_t chunk = slice * S + c;
  const int doc = valid ? a.chunk_doc[chunk] : -1;
  const bool live = doc >= 0;
  const bool multi = live && a.chunk_multi[chunk];
  const float a0 = AIR ? a.alpha : 0.f;
  const float alpha = a.alpha;

  for (int k = lane; k < KR; k += oni::kWave) bt[k] = t.b[k];
  cdoc[lane] = doc;
  cmul[lane] = multi ? 1 : 0;
  for (int k = 0; k < KR; k += 4) {
    int4 v = make_int4(0, 0, 0, 0);
    if (live) v = *reinterpret_cast<const int4*>(a.ndk_src + (int64_t)doc * KS + k);
    row[(k + 0) * 64 + lane] = (float)v.x + a0;
    row[(k + 1) * 64 + lane] = (float)v.y + a0;
    row[(k + 2) * 64 + lane] = (float)v.z + a0;
    row[(k + 3) * 64 + lane] = (float)v.w + a0;
  }
  __syncthreads();
  float R = 0.f;
  for (int k = 0; k < K; ++k) {
    const float rv = row[k * 64 + lane];
    R = fmaf(AIR ? rv : rv + alpha, bt[k], R);
  }

  const int steps = a.slice_len[slice0];  // slice0 < n_slices: the grid covers the slices exactly
  const int len = valid ? a.slice_len[slice] : 0;
  const int64_t off = valid ? a.slice_off[slice] : 0;
  const uint32_t key = live ? a.chunk_key[chunk] : 0u;
  const uint32_t pos0 = live ? (uint32_t)a.chunk_pos0[chunk] : 0u;
  const uint32_t sweep = *a.sweep_ctr;

  oni::U4 r{0, 0, 0, 0};
  // ping-pong word lists: the list of token s+1's word is fetched into the other buffer while step
  // s samples (its word id streams two steps ahead), so a word change never waits on a gather
  float la_b[2][kWsE];
  uint32_t lk_b[2][kWsE / 4];
  int L_b[2] = {0, 0};
#pragma unroll
  for (int j = 0; j < kWsE; ++j) la_b[0][j] = la_b[1][j] = 0.f;
#pragma unroll
  for (int j = 0; j < kWsE / 4; ++j) lk_b[0][j] = lk_b[1][j] = 0u;
  const int EL = KS < kWsE ? KS : kWsE;  // entries a row holds (uniform): loads never leave the row
  auto load_list = [&](auto PC, uint32_t w) {
    constexpr int P = decltype(PC)::value;
    if (w == oni::kPadWord) return;
    L_b[P] = t.llen[w];
    const float* lap = t.la + (int64_t)w * KS;
    const uint32_t* lkp = reinterpret_cast<const uint32_t*>(t.lk + (int64_t)w * KS);
#pragma unroll
    for (int j = 0; j < kWsE; j += 4) {
      if (j < EL) {
        const float4 v = *reinterpret_cast<const float4*>(lap + j);
        la_b[P][j] = v.x; la_b[P][j + 1] = v.y; la_b[P][j + 2] = v.z; la_b[P][j + 3] = v.w;
        lk_b[P][j / 4] = lkp[j / 4];
      }
    }
  };
  int nchg = 0;
  uint32_t w0 = len > 0 ? a.tok_word[off + c] : oni::kPadWord;
  int z0 = len > 0 ? (int)a.tok_z[off + c] : 0;
  uint32_t w1 = len > 1 ? a.tok_word[off + S + c] : oni::kPadWord;
  int z1 = len > 1 ? (int)a.tok_z[off + S + c] : 0;
  load_list(std::integral_constant<int, 0>{}, w0);
  auto step = [&](auto PC, int s) {
    constexpr int P = decltype(PC)::value;
    const int64_t idx = off + (int64_t)s * S + c;
    const uint32_t w = w0;
    const int zo = z0;
    load_list(std::integral_constant<int, 1 - P>{}, w1);
    w0 = w1;
    z0 = z1;
    w1 = oni::kPadWord;
    if (s + 2 < len) {
      w1 = a.tok_word[idx + 2 * S];
      z1 = (int)a.tok_z[idx + 2 * S];
    }
    const float* la_r = la_b[P];
    const uint32_t* lk_r = lk_b[P];
    const int L = L_b[P];
    const bool act = w != oni::kPadWord;
    bool changed = false;
    if (act) {
      const uint32_t pos = pos0 + (uint32_t)s;
      if (s == 0 || (pos & 3u) == 0u) r = oni::philox10(oni::U4{pos >> 2, key, sweep, 1u}, a.seed0, a.seed1);
      const uint32_t rr = oni::pick4(r, pos & 3u);
      // count updates are LDS atomics without return (ds_add_f32): no round trip on the chain;
      // LDS executes a wave's operations in order, so the reads below see the decrement
      atomicAdd(&row[zo * 64 + lane], -1.0f);
      const float bzo = bt[zo];
      const int Lc = L < kWsE ? L : kWsE;
      // every count the word bucket needs is read before the first fma: one LDS round trip
      float v[kWsE];
#pragma unroll
      for (int j = 0; j < kWsE; j += 4) {
        if (!__ballot(j < Lc)) break;  // uniform over the active lanes; independent of loaded data
        const uint32_t kq = lk_r[j / 4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) v[j + jj] = j + jj < Lc ? row[((kq >> (8 * jj)) & 0xFFu) * 64 + lane] : 0.f;
      }
      R = R - bzo;
      float cum[kWsE];
      float W = 0.f;
#pragma unroll
      for (int j = 0; j < kWsE; j += 4) {
        if (!__ballot(j < Lc)) break;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          if (j + jj < Lc) W = fmaf(AIR ? v[j + jj] : v[j + jj] + alpha, la_r[j + jj], W);
          cum[j + jj] = W;
        }
      }
      const float* lap = t.la + (int64_t)w * KS;
      const uint8_t* lkp = t.lk + (int64_t)w * KS;
      for (int j = kWsE; j < L; ++j) {  // slow path: lists longer than the register capacity
        const float rv = row[(int)lkp[j] * 64 + lane];
        W = fmaf(AIR ? rv : rv + alpha, lap[j], W);
      }
      const float thr = oni::u01(rr) * (W + R);
      if (t.stats) {
        const uint64_t sm = __ballot(!(thr < W)), sl = __ballot(L > kWsE), all = __ballot(true);
        int mx = Lc;
#pragma unroll
        for (int m = 1; m < oni::kWave; m <<= 1) mx = max(mx, __shfl_xor(mx, m));
        if (lane == __ffsll((unsigned long long)all) - 1) {
          atomicAdd(&t.stats[0], (unsigned long long)__popcll(all));
          atomicAdd(&t.stats[1], (unsigned long long)__popcll(sm));
          atomicAdd(&t.stats[2], (unsigned long long)__popcll(sl));
          atomicAdd(&t.stats[3], (unsigned long long)mx);
          atomicAdd(&t.stats[4], 1ull);
        }
      }
      int zn = -1;
      if (thr < W) {
#pragma unroll
        for (int j = 0; j < kWsE; j += 4) {
          if (!__ballot(j < Lc)) break;
          const uint32_t kq = lk_r[j / 4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            if (zn < 0 && j + jj < Lc && cum[j + jj] > thr) zn = (int)((kq >> (8 * jj)) & 0xFFu);
        }
        if (zn < 0) {
          float W2 = cum[kWsE - 1];
          for (int j = kWsE; j < L; ++j) {
            const int kk = (int)lkp[j];
            const float rv = row[kk * 64 + lane];
            W2 = fmaf(AIR ? rv : rv + alpha, lap[j], W2);
            if (W2 > thr) {
              zn = kk;
              break;
            }
          }
          if (zn < 0) zn = (int)lkp[L - 1];  // unreachable: W2 ends at W > thr
        }
      } else {
        // smoothing bucket: walk the fma chain over all topics, eight LDS reads in flight at a time
        const float tt = thr - W;
        float acc = 0.f;
        zn = K - 1;
        for (int k0 = 0; k0 < K; k0 += 8) {
          float rv[8], bv[8];
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            rv[jj] = k0 + jj < K ? row[(k0 + jj) * 64 + lane] : 0.f;
            bv[jj] = k0 + jj < K ? bt[k0 + jj] : 0.f;
          }
          bool hit = false;
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            if (!hit && k0 + jj < K) {
              acc = fmaf(AIR ? rv[jj] : rv[jj] + alpha, bv[jj], acc);
              if (acc > tt) {
                zn = k0 + jj;
                hit = true;
              }
            }
          }
          if (hit) break;
        }
      }
      atomicAdd(&row[zn * 64 + lane], 1.0f);
      R = R + bt[zn];
      changed = zn != zo;
      if (changed) {
        ++nchg;
        a.tok_z[idx] = (uint8_t)zn;
        if constexpr (MODE == 3) a.z_w[a.wpos[idx]] = (uint8_t)zn;
        if constexpr (MODE == 4) mark_changed_w(a, a.wpos[idx], zo, zn);
        if constexpr (MODE == 1) {
          atomicAdd(&a.dnwk[(int64_t)w * KS + zo], -1);
          atomicAdd(&a.dnwk[(int64_t)w * KS + zn], 1);
        }
      }
    }
    if constexpr (MODE == 2) {
      // one u64 per SELL step of each slice, bit c*G for chunk c (the dense samplers' layout);
      // chunk 0 of a slice is its longest, so it is active at every step of that slice
      const uint64_t m = __ballot(changed);
      if (c == 0 && s < len) {
        const uint64_t mine = (m >> (sq * S)) & (S == 64 ? ~0ull : ((1ull << S) - 1ull));
        uint64_t spread = 0;
        for (int i = 0; i < S; ++i) spread |= ((mine >> i) & 1ull) << (i * G);
        a.chg_mask[(off + (int64_t)s * S) / S] = spread;
      }
    }
  };
  for (int s = 0; s < steps; s += 2) {
    step(std::integral_constant<int, 0>{}, s);
    if (s + 1 < steps) step(std::integral_constant<int, 1>{}, s + 1);
  }
  if (a.chg_count) add_wave_count(a.chg_count, nchg);

  // ---- epilogue: doc rows, split-document deltas, per-topic totals ---------------------------
  // Each lane turns its row into Δ = n_final - n_start (stored back in LDS as int bits) and
  // writes its full row if the doc is not split over chunks; then lane k walks topic k over the
  // 64 chunks, summing runs of chunks of one split doc (adjacent in the slice) into ONE atomic
  // per run, and the slice's Δn_k into one atomic per topic.
  int32_t* rowi = reinterpret_cast<int32_t*>(row);
  for (int k = 0; k < KR; k += 4) {
    int4 n0 = make_int4(0, 0, 0, 0);
    if (live) n0 = *reinterpret_cast<const int4*>(a.ndk_src + (int64_t)doc * KS + k);
    const int n1x = (int)(row[(k + 0) * 64 + lane] - a0), n1y = (int)(row[(k + 1) * 64 + lane] - a0);
    const int n1z = (int)(row[(k + 2) * 64 + lane] - a0), n1w = (int)(row[(k + 3) * 64 + lane] - a0);
    if (live && !multi) *reinterpret_cast<int4*>(a.ndk_dst + (int64_t)doc * KS + k) = make_int4(n1x, n1y, n1z, n1w);
    rowi[(k + 0) * 64 + lane] = live ? n1x - n0.x : 0;
    rowi[(k + 1) * 64 + lane] = live ? n1y - n0.y : 0;
    rowi[(k + 2) * 64 + lane] = live ? n1z - n0.z : 0;
    rowi[(k + 3) * 64 + lane] = live ? n1w - n0.w : 0;
  }
  if (live && !multi)
    for (int k = KR; k < KS; k += 4) *reinterpret_cast<int4*>(a.ndk_dst + (int64_t)doc * KS + k) = make_int4(0, 0, 0, 0);
  __syncthreads();
  const int rep = (int)(blockIdx.x & (unsigned)(a.nk_rep - 1));
  for (int k = lane; k < K; k += oni::kWave) {
    int tot = 0, run = 0;
    for (int c = 0; c < oni::kWave; ++c) {
      const int d = rowi[k * 64 + c];
      tot += d;
      if (cmul[c]) {
        run += d;
        if (c == oni::kWave - 1 || cdoc[c + 1] != cdoc[c] || !cmul[c + 1]) {
          if (run) atomicAdd(a.ndk_dst + (int64_t)cdoc[c] * KS + k, run);
          run = 0;
        }
      }
    }
    if (tot) atomicAdd(&a.dnk[rep * KS + k], tot);
  }
}

// ---- word-sparse sampler on G-lane units (K > 32) --------------------------------------------
// k_gibbs_ws holds a whole doc row per lane in LDS (26 KB per 64 chains at K = 100: 6 waves per
// CU, and the measured kernel was slower than the dense one). Here the layout is the dense LDS
// sampler's (k_gibbs_ldsg): unit = G lanes, lane g owns topics [g·KP, (g+1)·KP) in its LDS row
// (20 waves per CU at K = 100), and the word bucket is split the same way -- lane g walks only the
// word's list entries in its topic range (contiguous in the ascending list; the per-word lane
// offsets come from k_ws_tables). Per lane: W_g over its entries, R_g its smoothing bucket (fma
// chain over its topics at chunk start, ± b on count changes), T_g = W_g + R_g combined by the
// same DPP Hillis-Steele scan as ldsg; the first lane with incl > thr draws inside its range.
// Numerics: oni355/ref/spec.py gibbs_pass_wsg (bitwise).
template <int G, int KP, int MODE, bool AIR>
__global__ __launch_bounds__(kBlock) void k_gibbs_wsg(const OniGibbs a, const OniWsTabs t) {
  static_assert(G > 1, "one-lane units use k_gibbs_ws");
  constexpr int S = oni::kWave / G;
  constexpr int KS = G * KP;
  constexpr int kSlots = LdsRow<KP>::kSlots;
  constexpr int E = 8;  // register capacity of a lane's share of the word's list
  __shared__ float4 sa[kBlock * kSlots];
  __shared__ float bt[KS];
  __shared__ int32_t red[kWavesPerBlock][KS];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int c = lane / G;
  const int g = lane % G;
  const int K = a.K;
  const int64_t slice = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const bool valid = slice < a.n_slices;
  const int64_t chunk = slice * S + c;
  const int doc = valid ? a.chunk_doc[chunk] : -1;
  const bool live = doc >= 0;
  const int kbase = g * KP;
  const float alpha = a.alpha;
  float4* row = sa + threadIdx.x * kSlots;
  float* rowf = reinterpret_cast<float*>(row);
  for (int k = threadIdx.x; k < KS; k += kBlock) bt[k] = t.b[k];
  {
    int32_t n0[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) n0[j] = 0;
    if (live) load_row_i<KP>(a.ndk_src + (int64_t)doc * KS + kbase, n0);
    const float a0 = AIR ? alpha : 0.f;
#pragma unroll
    for (int j = 0; j < KP / 4; ++j)
      row[j] = make_float4((float)n0[4 * j] + a0, (float)n0[4 * j + 1] + a0, (float)n0[4 * j + 2] + a0,
                           (float)n0[4 * j + 3] + a0);
  }
  __syncthreads();
  float R = 0.f;
#pragma unroll
  for (int j = 0; j < KP; ++j) R = fmaf(AIR ? rowf[j] : rowf[j] + alpha, bt[kbase + j], R);

  const int len = valid ? a.slice_len[slice] : 0;
  const int64_t off = valid ? a.slice_off[slice] : 0;
  const uint32_t key = live ? a.chunk_key[chunk] : 0u;
  const uint32_t pos0 = live ? (uint32_t)a.chunk_pos0[chunk] : 0u;
  const uint32_t sweep = *a.sweep_ctr;
  constexpr int kRefresh = 4 * G - 3;  // wave-uniform Philox refresh, as k_gibbs_ldsg
  uint32_t gbase = pos0 >> 2;
  oni::U4 r = oni::philox10(oni::U4{gbase + (uint32_t)g, key, sweep, 1u}, a.seed0, a.seed1);
  int next_refresh = kRefresh;
  uint32_t wcur = oni::kPadWord;
  int jb = 0, nb = 0;
  float la_r[E];
  int lk_r[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    la_r[j] = 0.f;
    lk_r[j] = 0;
  }
  int nchg = 0;
  uint32_t w_nx = len > 0 ? a.tok_word[off + c] : oni::kPadWord;
  int z_nx = len > 0 ? (int)a.tok_z[off + c] : 0;
  for (int s = 0; s < len; ++s) {
    const int64_t idx = off + (int64_t)s * S + c;
    const uint32_t w = w_nx;
    const int zo = z_nx;
    if (s + 1 < len) {
      w_nx = a.tok_word[idx + S];
      z_nx = a.tok_z[idx + S];
    }
    if (s == next_refresh) {
      next_refresh += kRefresh;
      gbase = (pos0 + (uint32_t)s) >> 2;
      r = oni::philox10(oni::U4{gbase + (uint32_t)g, key, sweep, 1u}, a.seed0, a.seed1);
    }
    if (w == oni::kPadWord) continue;  // uniform across the G lanes of a unit
    const uint32_t pos = pos0 + (uint32_t)s;
    const uint32_t gi = pos >> 2;
    const uint32_t rr = (uint32_t)__shfl((int)oni::pick4(r, pos & 3u), (int)(gi - gbase), G);
    const float* lap = t.la + (int64_t)w * KS;
    const uint8_t* lkp = t.lk + (int64_t)w * KS;
    if (w != wcur) {  // this lane's share of the word's list: entries [jb, jb + nb)
      const uint32_t lo = t.lofs[w];
      const int L = t.llen[w];
      jb = (int)((lo >> (8 * g)) & 0xFFu);
      const int je = g + 1 < G ? (int)((lo >> (8 * (g + 1))) & 0xFFu) : L;
      nb = je - jb;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        if (j < nb) {
          la_r[j] = lap[jb + j];
          lk_r[j] = (int)lkp[jb + j] - kbase;
        }
      }
      wcur = w;
    }
    const unsigned zlo = (unsigned)(zo - kbase);
    if (zlo < (unsigned)KP) {
      atomicAdd(&rowf[zlo], -1.0f);
      R = R - bt[zo];
    }
    const int nr = nb < E ? nb : E;
    float v[E];
#pragma unroll
    for (int j = 0; j < E; ++j) v[j] = j < nr ? rowf[lk_r[j]] : 0.f;
    float cum[E];
    float W = 0.f;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      if (j < nr) W = fmaf(AIR ? v[j] : v[j] + alpha, la_r[j], W);
      cum[j] = W;
    }
    for (int j = E; j < nb; ++j) {  // slow path: a longer share than the register capacity
      const float rv = rowf[(int)lkp[jb + j] - kbase];
      W = fmaf(AIR ? rv : rv + alpha, lap[jb + j], W);
    }
    const float T = W + R;
    const float incl = group_scan_dpp<G>(T, g);
    float excl = dpp_row_shr<1>(incl);
    if (g == 0) excl = 0.f;
    const float total = __shfl(incl, G - 1, G);
    const float thr = oni::u01(rr) * total;
    int gs = group_sum_dpp<G>(incl <= thr ? 1 : 0);
    gs = gs < G - 1 ? gs : G - 1;
    int z = 0;
    if (g == gs) {
      const float tt = thr - excl;
      if (tt < W) {
        int pick = -1;
#pragma unroll
        for (int j = 0; j < E; ++j)
          if (pick < 0 && j < nr && cum[j] > tt) pick = j;
        if (pick < 0) {
          float W2 = nr > 0 ? cum[nr - 1] : 0.f;
          for (int j = E; j < nb; ++j) {
            const float rv = rowf[(int)lkp[jb + j] - kbase];
            W2 = fmaf(AIR ? rv : rv + alpha, lap[jb + j], W2);
            if (W2 > tt) {
              pick = j;
              break;
            }
          }
          if (pick < 0) pick = nb - 1;  // unreachable in exact arithmetic: W2 ends at W > tt
        }
        z = kbase + (pick < E ? lk_r[pick] : (int)lkp[jb + pick] - kbase);
      } else {
        const float t2 = tt - W;
        const int kend = K - kbase < KP ? K - kbase : KP;
        float acc = 0.f;
        z = kbase + kend - 1;
        for (int j = 0; j < kend; ++j) {
          acc = fmaf(AIR ? rowf[j] : rowf[j] + alpha, bt[kbase + j], acc);
          if (acc > t2) {
            z = kbase + j;
            break;
          }
        }
      }
    }
    const int zn = __shfl(z, gs, G);
    const unsigned znl = (unsigned)(zn - kbase);
    if (znl < (unsigned)KP) {
      atomicAdd(&rowf[znl], 1.0f);
      R = R + bt[zn];
    }
    const bool changed = zn != zo && g == 0;
    if (changed) {
      ++nchg;
      a.tok_z[idx] = (uint8_t)zn;
      if constexpr (MODE == 3) a.z_w[a.wpos[idx]] = (uint8_t)zn;
      if constexpr (MODE == 4) mark_changed_w(a, a.wpos[idx], zo, zn);
      if constexpr (MODE == 1) {
        atomicAdd(&a.dnwk[(int64_t)w * KS + zo], -1);
        atomicAdd(&a.dnwk[(int64_t)w * KS + zn], 1);
      }
    }
    if constexpr (MODE == 2) {
      const uint64_t m = __ballot(changed);
      if (lane == 0) a.chg_mask[(off + (int64_t)s * S) / S] = m;
    }
  }
  if (a.chg_count) add_wave_count(a.chg_count, nchg);
  // ---- epilogue (as k_gibbs_ldsg): doc rows + per-topic totals --------------------------------
  int32_t d[KP], n[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    n[j] = (int32_t)(AIR ? rowf[j] - alpha : rowf[j]);
    d[j] = 0;
  }
  if (live) {
    int32_t* dst = a.ndk_dst + (int64_t)doc * KS + kbase;
    int32_t n0[KP];
    load_row_i<KP>(a.ndk_src + (int64_t)doc * KS + kbase, n0);
#pragma unroll
    for (int j = 0; j < KP; ++j) d[j] = n[j] - n0[j];
    if (!a.chunk_multi[chunk]) {
#pragma unroll
      for (int j = 0; j < KP; j += 4) *reinterpret_cast<int4*>(dst + j) = make_int4(n[j], n[j + 1], n[j + 2], n[j + 3]);
    }
  }
  {
    const bool multi = live && a.chunk_multi[chunk];
    if (__ballot(multi)) flush_multi_rows<G, KP>(a.ndk_dst, KS, doc, multi, kbase, d);
  }
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    int vv = d[j];
#pragma unroll
    for (int m = G; m < oni::kWave; m <<= 1) vv += __shfl_xor(vv, m);
    d[j] = vv;
  }
  if (c == 0) {
#pragma unroll
    for (int j = 0; j < KP; ++j) red[wave][kbase + j] = d[j];
  }
  __syncthreads();
  if (threadIdx.x < KS) {
    int vv = 0;
#pragma unroll
    for (int w2 = 0; w2 < kWavesPerBlock; ++w2) vv += red[w2][threadIdx.x];
    if (vv) atomicAdd(&a.dnk[(int)(blockIdx.x & (unsigned)(a.nk_rep - 1)) * KS + threadIdx.x], vv);
  }
}

template <int G, int KP>
int launch_wsg(const OniGibbs& a, const OniWsTabs& t, int mode, hipStream_t s) {
  const unsigned grid = (unsigned)((a.n_slices + kWavesPerBlock - 1) / kWavesPerBlock);
  if (grid == 0) return 0;
  const bool air = (a.flags & 1) != 0;
#define ONI_WSG(m_)                                                          \
  if (air) k_gibbs_wsg<G, KP, m_, true><<<grid, kBlock, 0, s>>>(a, t);       \
  else k_gibbs_wsg<G, KP, m_, false><<<grid, kBlock, 0, s>>>(a, t);
  switch (mode) {
    case 0: ONI_WSG(0) break;
    case 1: ONI_WSG(1) break;
    case 2: ONI_WSG(2) break;
    case 3: ONI_WSG(3) break;
    default: ONI_WSG(4) break;
  }
#undef ONI_WSG
  return (int)hipGetLastError();
}

// Per-sweep tables of k_gibbs_ws from the refreshed counts: one wave per word compacts the
// topics with n_wk > 0 (ballot + prefix popcount, ascending k) with a_wk = n_wk / (n_k + Vβ);
// block 0 writes b_k = β / (n_k + Vβ). den_k is the same f32 expression as k_apply's.
__global__ __launch_bounds__(256) void k_ws_tables(const int32_t* __restrict__ nwk, const int32_t* __restrict__ nk,
                                                   int64_t V, int K, int KS, float beta, float vbeta,
                                                   int32_t* __restrict__ llen, uint8_t* __restrict__ lk,
                                                   float* __restrict__ la, float* __restrict__ b,
                                                   uint32_t* __restrict__ lofs, int G, int KP) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  if (blockIdx.x == 0)
    for (int k = threadIdx.x; k < KS; k += blockDim.x) b[k] = k < K ? beta / ((float)nk[k] + vbeta) : 0.f;
  for (int64_t w = wave0; w < V; w += nwaves) {
    int base = 0;
    uint32_t offs = 0;  // byte g: entries with topic < g·KP (lane g's first entry)
    for (int k0 = 0; k0 < K; k0 += oni::kWave) {
      const int k = k0 + lane;
      const int32_t n = k < K ? nwk[w * KS + k] : 0;
      const uint64_t m = __ballot(n > 0);
      if (n > 0) {
        const int p = base + __popcll(m & ((1ull << lane) - 1ull));
        lk[w * KS + p] = (uint8_t)k;
        la[w * KS + p] = (float)n / ((float)nk[k] + vbeta);
      }
      for (int gg = 1; gg < G; ++gg) {
        const int lim = gg * KP - k0;  // lanes of this block below the lane boundary
        const uint64_t below = lim <= 0 ? 0ull : (lim >= 64 ? ~0ull : ((1ull << lim) - 1ull));
        offs += (uint32_t)__popcll(m & below) << (8 * gg);
      }
      base += __popcll(m);
    }
    if (lane == 0) {
      llen[w] = base;
      if (lofs) lofs[w] = offs;
    }
  }
}

}  // namespace

ONI_API int oni_gibbs_ws_launch(const OniGibbs* a, const OniWsTabs* t, int G, int mode, hipStream_t s) {
  if (G != 1 && G != 2 && G != 4 && G != 8 && G != 16) return (int)hipErrorInvalidValue;
  if (a->K < 1 || a->K > 240 || a->K > a->KS || a->KS % 4 || mode < 0 || mode > 4) return (int)hipErrorInvalidValue;
  if (a->nk_rep < 1 || (a->nk_rep & (a->nk_rep - 1))) return (int)hipErrorInvalidValue;
  if (mode == 2 && !a->chg_mask) return (int)hipErrorInvalidValue;
  if (mode == 3 && (!a->wpos || !a->z_w)) return (int)hipErrorInvalidValue;
  if (mode == 4 && (!a->wpos || !a->zz_w || !a->chg_mask)) return (int)hipErrorInvalidValue;
  if (!t->llen || !t->lk || !t->la || !t->b) return (int)hipErrorInvalidValue;
  if (a->n_slices <= 0) return 0;
  const int KR = (a->K + 3) / 4 * 4;
  const size_t lds = ((size_t)KR * 64 + KR + 128) * 4;
  const unsigned grid = (unsigned)((a->n_slices + G - 1) / G);
  const bool air = (a->flags & 1) != 0;
#define ONI_WS(m_)                                                                   \
  if (air) k_gibbs_ws<m_, true><<<grid, 64, lds, s>>>(*a, *t, KR, G);                   \
  else k_gibbs_ws<m_, false><<<grid, 64, lds, s>>>(*a, *t, KR, G);
  switch (mode) {
    case 0: ONI_WS(0) break;
    case 1: ONI_WS(1) break;
    case 2: ONI_WS(2) break;
    case 3: ONI_WS(3) break;
    default: ONI_WS(4) break;
  }
#undef ONI_WS
  return (int)hipGetLastError();
}

ONI_API int oni_ws_tables(const int32_t* nwk, const int32_t* nk, int64_t V, int K, int KS, float beta, float vbeta,
                          int32_t* llen, uint8_t* lk, float* la, float* b, uint32_t* lofs, int G, int KP,
                          hipStream_t s) {
  if (K < 1 || K > 240 || K > KS || KS % 4) return (int)hipErrorInvalidValue;
  if (lofs && (G < 1 || G > 4 || G * KP != KS)) return (int)hipErrorInvalidValue;
  const int64_t waves = V > 0 ? V : 1;
  k_ws_tables<<<oni::grid_for(waves * 64, 256, 4096), 256, 0, s>>>(nwk, nk, V, K, KS, beta, vbeta, llen, lk, la, b,
                                                                    lofs, lofs ? G : 1, KP);
  return (int)hipGetLastError();
}

ONI_API int oni_gibbs_wsg_launch(const OniGibbs* a, const OniWsTabs* t, int G, int KP, int mode, hipStream_t s) {
  if (a->K < 1 || a->K > a->KS || a->KS != G * KP || mode < 0 || mode > 4) return (int)hipErrorInvalidValue;
  if (a->nk_rep < 1 || (a->nk_rep & (a->nk_rep - 1))) return (int)hipErrorInvalidValue;
  if (mode == 2 && !a->chg_mask) return (int)hipErrorInvalidValue;
  if (mode == 3 && (!a->wpos || !a->z_w)) return (int)hipErrorInvalidValue;
  if (mode == 4 && (!a->wpos || !a->zz_w || !a->chg_mask)) return (int)hipErrorInvalidValue;
  if (!t->llen || !t->lk || !t->la || !t->b || !t->lofs) return (int)hipErrorInvalidValue;
#define ONI_CASE(g_, kp_) \
  if (G == g_ && KP == kp_) return launch_wsg<g_, kp_>(*a, *t, mode, s);
  ONI_CASE(2, 20) ONI_CASE(2, 24) ONI_CASE(2, 28) ONI_CASE(4, 16) ONI_CASE(4, 20) ONI_CASE(4, 24) ONI_CASE(4, 28)
#undef ONI_CASE
  return (int)hipErrorInvalidValue;
}
