// Collapsed-Gibbs sweep kernels (K10) and their launcher template, shared by gibbs.hip and the
// per-unit-width instantiation units gibbs_g*.hip (compiled in parallel).
#pragma once
// K10/K11/K12 -- collapsed-Gibbs LDA on CDNA4: init, sweep, delta-apply (+ q-table refresh).
//
// Replaces oni-lda-c's variational-EM `lda est` E-step/M-step loop (lda-estimate.c run_em /
// doc_e_step, lda-inference.c, lda-model.c lda_mle; SURVEY.md §3.2, [U-H]) with collapsed Gibbs
// sampling, as the north star requires (BASELINE.json).
//
// The conditional ("remove its old z"): a token of word w in doc d whose
// topic is zo draws topic k with weight
//
//     p_k ∝ (n_dk^¬t + α) · (n_wk^¬t + β)/(n_k^¬t + Vβ)
//
// with the token removed from BOTH sides. The doc side is exact within a chunk (the unit holds the
// doc's counts and updates them token by token). The word side is the sweep-start snapshot
// q[w,k] = (n_wk+β)/(n_k+Vβ) (AD-LDA staleness, one snapshot per sweep), which still counts the
// token at its sweep-start topic zo; so topic zo's factor is replaced by
//     q' = (n_wzo − 1 + β)/(D_zo − 1) = fma(q_zo, A_zo, −B_zo),  D = n_k + Vβ,
// A = D/(D−1), B = 1/(D−1) (per-topic sweep constants written by k_apply next to q, `qfix`).
// Numerics are pinned and replayed bit for bit by oni355/ref/spec.py gibbs_pass.
//
// Execution model (MI355X-first):
//  * Documents (IPs) are owned by sampler "units" of G lanes; a unit walks one chunk (≤ L tokens of
//    one doc) sequentially holding the doc's topic counts (KP per lane, KS = G*KP padded topics).
//  * A wave = one SELL slice of S = 64/G chunks; tokens are step-major so per-step word/topic
//    loads are coalesced.
//  * G = 1 for K ≤ 32 (k_gibbs_x1: one lane owns all topics, counts in registers); G ∈ {2, 4, 8,
//    16} above (k_gibbs_ldsg: counts in LDS, DPP scans across the unit).
//  * Draws are Philox4x32-10 keyed by (seed) with counter (pos/4, doc key, sweep, stream): the
//    chain is a pure function of the data + seed — bitwise identical for any GPU count, shard
//    plan, chunk packing or resume point.
//  * Long documents span several chunks. Those chunks start from the sweep-start row of ndk_src
//    and add their deltas into ndk_dst (pre-copied row), with integer atomics: still order-free.
#include "oni_common.h"

struct OniGibbs {
  const uint32_t* tok_word;    // SELL [Σ slice_len*S]
  uint8_t* tok_z;              // SELL
  const int64_t* slice_off;    // [n_slices]
  const int32_t* slice_len;    // [n_slices]
  const int32_t* chunk_doc;    // [n_slices*S] local doc row, -1 = padding chunk
  const int32_t* chunk_pos0;   // position of the chunk's first token inside its doc
  const uint32_t* chunk_key;   // doc key (RNG stream id; global, shard-independent)
  const uint8_t* chunk_multi;  // 1 if the doc is split over several chunks
  const int32_t* ndk_src;      // [D][KS] sweep-start doc-topic counts
  int32_t* ndk_dst;            // [D][KS] output doc-topic counts
  const float* q;              // [V][KS] sweep-start word factor
  const float* qfix;           // [2][KS] token-exclusion constants: A (row 0), B (row 1)
  int32_t* dnwk;               // [V][KS] word-topic delta (init: the n_wk table itself)
  int32_t* dnk;                // [nk_rep][KS] topic-total delta replicas (init: n_k itself, nk_rep = 1)
  const uint32_t* sweep_ctr;   // device scalar: current sweep number (≥ 1), graph-replay safe
  uint64_t* chg_mask;          // MODE 2: one u64 per SELL step, bit c*G set if slot c's topic changed
  const int32_t* wpos;         // MODE 3/4: word-sorted position of every SELL slot
  uint8_t* z_w;                // MODE 3: topic array in word-sorted order (kept in sync for changed tokens)
  uint32_t* zz_w;              // MODE 4, word-sorted [T]: bits 0-15 (old | new << 8) topics of a changed
                                //   token; bits 16-31 its word's row in its k_wdelta_recount block
                                //   (written once with the corpus, 0xFFFF: read wsorted)
                               // (MODE 4 reuses chg_mask as a u32 bitmap over word-sorted positions)
  int32_t* chg_count;          // optional: += number of tokens whose topic changed (drives the auto mode)
  const int32_t* exact_guard;  // optional device flag (1: every count this sweep's rows can reach keeps
                               //   n + α exact in f32): the row-f32 kernels run when it is set, the generic
                               //   kernel (launched beside them) when it is not -- see k_exact_guard
  uint8_t* tok_zlag;           // optional, SELL (ONI_X01_LAG): the topic each token holds in the counts
                               //   behind q (one sweep older than the doc rows): the word-side exclusion
                               //   is taken there; the pass writes tok_zlag := the token's sweep-start topic
  int64_t n_slices;
  int32_t K;
  int32_t KS;
  float alpha;
  uint32_t seed0, seed1;
  int32_t nk_rep;              // dnk holds nk_rep replicas of [KS] (power of 2): block b adds into b % nk_rep
  int32_t flags;               // bit 0: n + α is exact in f32 for every count of this corpus (rows may hold it);
                               // bits 1-2: kernel A/B variants; bit 3: init pass puts every token of a word
                               // in topic ⌊mix32(w)·K / 2^32⌋ (seed-free start)
};

namespace {

constexpr int kBlock = 256;
// Δ buffers are [V·KS | nk_rep·KS | kDnAux]: the aux words ride along in the all-reduce
// ([0] = number of changed tokens this sweep); k_apply zeroes all of it in the other buffer.
constexpr int kDnAux = 4;
constexpr int kWavesPerBlock = kBlock / oni::kWave;

template <int KP>
__device__ __forceinline__ void load_row_i(const int32_t* __restrict__ p, int32_t (&v)[KP]) {
#pragma unroll
  for (int j = 0; j < KP; j += 4) {
    const int4 t = *reinterpret_cast<const int4*>(p + j);
    v[j] = t.x; v[j + 1] = t.y; v[j + 2] = t.z; v[j + 3] = t.w;
  }
}
template <int KP>
__device__ __forceinline__ void load_row_f(const float* __restrict__ p, float (&v)[KP]) {
#pragma unroll
  for (int j = 0; j < KP; j += 4) {
    const float4 t = *reinterpret_cast<const float4*>(p + j);
    v[j] = t.x; v[j + 1] = t.y; v[j + 2] = t.z; v[j + 3] = t.w;
  }
}

// Sum a per-lane count over the wave; lane 0 adds it to *dst (one atomic per wave).
__device__ __forceinline__ void add_wave_count(int32_t* dst, int v) {
#pragma unroll
  for (int m = 1; m < oni::kWave; m <<= 1) v += __shfl_xor(v, m);
  if ((threadIdx.x & (oni::kWave - 1)) == 0 && v) atomicAdd(dst, v);
}

// Long documents: all full-length chunks of a doc are adjacent in the chunk order (stable sort by
// length), so consecutive units of a wave often belong to the same doc. Their count deltas are
// summed over each such run inside the wave first (segmented suffix sum over units, shuffles at
// unit stride G) and only the run's first unit issues the atomics: same-address atomics execute
// serially at the memory side, so one heavy IP spread over thousands of chunks would otherwise
// queue KS × chunks adds on a single row.
template <int G, int KP>
__device__ __forceinline__ void flush_multi_rows(int32_t* __restrict__ ndk_dst, int KS, int doc, bool multi,
                                                 int kbase, const int32_t (&delta)[KP]) {
  constexpr int S = oni::kWave / G;
  const int lane = threadIdx.x & (oni::kWave - 1);
  const int c = lane / G;
  const int prev_doc = __shfl_up(doc, G);
  const bool head = (c == 0) || prev_doc != doc;
  const uint64_t heads = __ballot(head && (lane % G) == 0);
  const int first_lane_of_next = c * G + G;
  const uint64_t above = first_lane_of_next < oni::kWave ? heads & (~0ull << first_lane_of_next) : 0ull;
  const int next = above ? (__ffsll((unsigned long long)above) - 1) / G : S;
  int32_t d[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) d[j] = delta[j];
#pragma unroll
  for (int off = 1; off < S; off <<= 1) {
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      const int o = __shfl_down(d[j], off * G);
      if (c + off < next) d[j] += o;
    }
  }
  if (multi && head) {
    int32_t* dst = ndk_dst + (int64_t)doc * KS + kbase;
#pragma unroll
    for (int j = 0; j < KP; ++j)
      if (d[j]) atomicAdd(dst + j, d[j]);
  }
}

// Epilogue shared by every sweep kernel: the unit's final doc counts n (KP per lane) → ndk_dst
// (single-chunk docs store the row, split docs add their delta), and the wave's / block's
// per-topic deltas → one dnk replica.
template <int G, int KP>
__device__ __forceinline__ void sweep_epilogue(const OniGibbs& a, int32_t (*red)[G * KP], int doc, bool live,
                                               int64_t chunk, int kbase, const int32_t (&n)[KP], bool init) {
  constexpr int KS = G * KP;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int c = lane / G;
  int32_t d[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) d[j] = 0;
  if (live) {
    int32_t* dst = a.ndk_dst + (int64_t)doc * KS + kbase;
    if (init) {
#pragma unroll
      for (int j = 0; j < KP; ++j) d[j] = n[j];
    } else {
      int32_t n0[KP];
      load_row_i<KP>(a.ndk_src + (int64_t)doc * KS + kbase, n0);
#pragma unroll
      for (int j = 0; j < KP; ++j) d[j] = n[j] - n0[j];
    }
    if (!a.chunk_multi[chunk]) {
#pragma unroll
      for (int j = 0; j < KP; j += 4) *reinterpret_cast<int4*>(dst + j) = make_int4(n[j], n[j + 1], n[j + 2], n[j + 3]);
    }
  }
  {
    const bool multi = live && a.chunk_multi[chunk];
    if (__ballot(multi)) flush_multi_rows<G, KP>(a.ndk_dst, KS, doc, multi, kbase, d);
  }
  // reduce d over the S units of this wave (lanes with equal g), then over the block's waves
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    int v = d[j];
#pragma unroll
    for (int m = G; m < oni::kWave; m <<= 1) v += __shfl_xor(v, m);
    d[j] = v;
  }
  if (c == 0) {
#pragma unroll
    for (int j = 0; j < KP; ++j) red[wave][kbase + j] = d[j];
  }
  __syncthreads();
  if (threadIdx.x < KS) {
    int v = 0;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) v += red[w][threadIdx.x];
    if (v) atomicAdd(&a.dnk[(int)(blockIdx.x & (unsigned)(a.nk_rep - 1)) * KS + threadIdx.x], v);
  }
}

// MODE 4: a changed token records (old, new) topic at its word-sorted position p and sets bit p
// of a word-sorted bitmap; k_wdelta_recount then visits only set bits.
__device__ __forceinline__ void mark_changed_w(const OniGibbs& a, int32_t p, int zo, int zn) {
  // one 2-B store into the low half (the row half stays): only read where the bit below is set
  reinterpret_cast<uint16_t*>(a.zz_w + p)[0] = (uint16_t)(zo | (zn << 8));
  atomicOr(reinterpret_cast<uint32_t*>(a.chg_mask) + (p >> 5), 1u << (p & 31));
}

// Philox blocks at a wave-uniform cadence for samplers with one chain per lane. A lane needs a
// new block whenever its token position enters a new 4-token group; with 64 chunks at random
// phases some lane does so on every step. Here every lane refreshes together every 4 steps and
// computes only the block of the group AFTER its current one (within a 4-step window a position
// lies in one of two consecutive groups): one block per lane per 4 steps, the same values.
struct PhiloxPair {
  oni::U4 cur, nxt;
  uint32_t pos0, key, sweep, stream;
  __device__ __forceinline__ void init(uint32_t p0, uint32_t k, uint32_t sw, uint32_t st, const OniGibbs& a) {
    pos0 = p0;
    key = k;
    sweep = sw;
    stream = st;
    nxt = oni::philox10(oni::U4{pos0 >> 2, key, sweep, stream}, a.seed0, a.seed1);
    cur = nxt;
  }
  // call with every s, before any lane-divergent exit (the refresh is wave-uniform)
  __device__ __forceinline__ void step(int s, const OniGibbs& a) {
    if ((s & 3) == 0) {
      cur = nxt;
      nxt = oni::philox10(oni::U4{((pos0 + (uint32_t)s) >> 2) + 1u, key, sweep, stream}, a.seed0, a.seed1);
    }
  }
  // chunk starts at multiples of 4 (flags bit 4: L % 4 == 0): a token's block is always `cur` and
  // its word index is s & 3 -- wave-uniform, so the pick is a scalar choice, not four selects
  __device__ __forceinline__ uint32_t pick_aligned(int s) const {
    switch (s & 3) {
      case 0: return cur.x;
      case 1: return cur.y;
      case 2: return cur.z;
      default: return cur.w;
    }
  }
  __device__ __forceinline__ uint32_t pick(int s) const {
    const uint32_t pos = pos0 + (uint32_t)s;
    const bool second = (pos >> 2) != ((pos0 + (uint32_t)(s & ~3)) >> 2);
    const uint32_t i = pos & 3u;
    // branch-free selects (v_cndmask): the value is lane-dependent
    const uint32_t x = second ? nxt.x : cur.x, y = second ? nxt.y : cur.y;
    const uint32_t z = second ? nxt.z : cur.z, w = second ? nxt.w : cur.w;
    const uint32_t lo = (i & 1u) ? y : x, hi = (i & 1u) ? w : z;
    return (i & 2u) ? hi : lo;
  }
};

// MODE: 0 = no n_wk bookkeeping (full recount afterwards), 1 = per-token Δ atomics,
//       2 = changed-slot ballot mask per step (delta recount afterwards),
//       3 = changed topics also scattered into the word-sorted copy z_w (streaming recount afterwards)
//       4 = changed tokens marked in a word-sorted bitmap + (old, new) topic copies (k_wdelta_recount)
// A changed token's bookkeeping is held back one step (issued after the next step's loads): every
// vector-memory op of a wave retires through one in-order vmcnt counter, so a store issued at the
// end of a step would make the next step's wait for its loads wait out the store as well.
template <int MODE>
struct Pend {
  bool on = false;
  int64_t idx = 0;
  int zo = 0, zn = 0;
  int32_t pw = 0;
  uint32_t w = 0;
  uint64_t m = 0;
  int64_t mi = -1;
  __device__ __forceinline__ void note(int64_t i, int o, int n, int32_t p, uint32_t ww) {
    on = true;
    idx = i;
    zo = o;
    zn = n;
    pw = p;
    w = ww;
  }
  __device__ __forceinline__ void flush(const OniGibbs& a, int KS) {
    if (on) {
      a.tok_z[idx] = (uint8_t)zn;
      if constexpr (MODE == 3) a.z_w[pw] = (uint8_t)zn;
      if constexpr (MODE == 4) mark_changed_w(a, pw, zo, zn);
      if constexpr (MODE == 1) {
        atomicAdd(&a.dnwk[(int64_t)w * KS + zo], -1);
        atomicAdd(&a.dnwk[(int64_t)w * KS + zn], 1);
      }
      on = false;
    }
    if constexpr (MODE == 2) {
      if (mi >= 0) a.chg_mask[mi] = m;
      mi = -1;
    }
  }
};

// ---- generic sampler: init pass + any-G fallback sweep ------------------------------------------
// Integer count rows in registers, q row loaded on a word change. Runs the init pass (uniform
// topics), and sweeps whenever the specialised kernels do not apply (n + α not exact in f32, e.g.
// α = 50/7). Numerics are the spec's: G = 1 replaces q_zo by q'; G > 1 scales the owner lane's
// weight of zo by f = q'/q_zo.
template <int G, int KP, bool INIT, int MODE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 8))) void k_gibbs(const OniGibbs a) {
  // flags bit 6: the guarded twin of a row-f32 kernel (launch_gibbs) -- it runs only when they do not
  if (!INIT && (a.flags & 64) && *a.exact_guard != 0) return;
  constexpr int S = oni::kWave / G;
  constexpr int KS = G * KP;
  __shared__ int32_t red[kWavesPerBlock][KS];

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int c = lane / G;
  const int g = lane % G;
  const int64_t slice = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const bool valid = slice < a.n_slices;
  const int64_t chunk = slice * S + c;
  const int doc = valid ? a.chunk_doc[chunk] : -1;
  const bool live = doc >= 0;
  const int kbase = g * KP;

  int32_t n[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) n[j] = 0;
  if (!INIT && live) load_row_i<KP>(a.ndk_src + (int64_t)doc * KS + kbase, n);

  const int len = valid ? a.slice_len[slice] : 0;
  const int64_t off = valid ? a.slice_off[slice] : 0;
  const uint32_t key = live ? a.chunk_key[chunk] : 0u;
  const uint32_t pos0 = live ? (uint32_t)a.chunk_pos0[chunk] : 0u;
  const uint32_t sweep = INIT ? 0u : *a.sweep_ctr;
  const uint32_t stream = INIT ? 0u : 1u;

  PhiloxPair rng;
  rng.init(pos0, key, sweep, stream, a);
  uint32_t wprev = oni::kPadWord;
  float qv[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) qv[j] = 0.f;
  int nchg = 0;
  constexpr bool WPF = !INIT && (MODE == 3 || MODE == 4);
  uint32_t w_nx = len > 0 ? a.tok_word[off + c] : oni::kPadWord;
  int z_nx = (!INIT && len > 0) ? (int)a.tok_z[off + c] : 0;
  int32_t p_nx = (WPF && len > 0) ? a.wpos[off + c] : 0;
  // lagged word side (ONI_X01_LAG): the word-side exclusion at the topic the counts behind q hold
  const bool lag = !INIT && a.tok_zlag != nullptr;
  int l_nx = (lag && len > 0) ? (int)a.tok_zlag[off + c] : z_nx;
  Pend<MODE> pend;
  for (int s = 0; s < len; ++s) {
    const int64_t idx = off + (int64_t)s * S + c;
    const uint32_t w = w_nx;
    const int zo = z_nx;
    const int zl = lag ? l_nx : zo;
    const int32_t pw = p_nx;
    if (s + 1 < len) {
      w_nx = a.tok_word[idx + S];
      if (!INIT) z_nx = (int)a.tok_z[idx + S];
      if (lag) l_nx = (int)a.tok_zlag[idx + S];
      if (WPF) p_nx = a.wpos[idx + S];
    }
    if constexpr (!INIT) pend.flush(a, KS);
    rng.step(s, a);
    if (w == oni::kPadWord) continue;  // uniform across the G lanes of a unit
    const uint32_t rr = rng.pick(s);
    if constexpr (INIT) {
      // flags bit 3: seed-free start, every token of a word in the word's hashed topic
      const int z = (int)__umulhi((a.flags & 8) ? oni::mix32(w) : rr, (uint32_t)a.K);
#pragma unroll
      for (int j = 0; j < KP; ++j) n[j] += (kbase + j == z);
      if (g == 0) {
        a.tok_z[idx] = (uint8_t)z;
        if (MODE == 1) atomicAdd(&a.dnwk[(int64_t)w * KS + z], 1);
      }
    } else {
#pragma unroll
      for (int j = 0; j < KP; ++j) n[j] -= (kbase + j == zo);
      if (w != wprev) {
        load_row_f<KP>(a.q + (int64_t)w * KS + kbase, qv);
        wprev = w;
      }
      const float qz = a.q[(int64_t)w * KS + zl];
      const float qe = fmaf(qz, a.qfix[zl], -a.qfix[KS + zl]);
      const float f = qe / qz;
      float loc[KP];
      float run = 0.f;
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        const bool own = kbase + j == zl;
        float av = (float)n[j] + a.alpha;
        float qj = qv[j];
        if (G == 1) qj = own ? qe : qj;
        else av = own ? av * f : av;
        run = fmaf(av, qj, run);
        loc[j] = run;
      }
      float excl = 0.f, total = run;
      if constexpr (G > 1) {
        float incl = run;
#pragma unroll
        for (int d = 1; d < G; d <<= 1) {
          const float y = __shfl_up(incl, d, G);
          if (g >= d) incl = incl + y;
        }
        excl = __shfl_up(incl, 1, G);
        if (g == 0) excl = 0.f;
        total = __shfl(incl, G - 1, G);
      }
      const float thr = oni::u01(rr) * total;
      int cnt = 0;
#pragma unroll
      for (int j = 0; j < KP; ++j) cnt += ((G > 1 ? excl + loc[j] : loc[j]) <= thr);
      if constexpr (G > 1) {
#pragma unroll
        for (int d = 1; d < G; d <<= 1) cnt += __shfl_xor(cnt, d, G);
      }
      const int zn = cnt < a.K - 1 ? cnt : a.K - 1;
#pragma unroll
      for (int j = 0; j < KP; ++j) n[j] += (kbase + j == zn);
      const bool changed = zn != zo && g == 0;
      if (changed) {
        ++nchg;
        pend.note(idx, zo, zn, pw, w);
      }
      if (lag && g == 0 && zl != zo) a.tok_zlag[idx] = (uint8_t)zo;
      if constexpr (MODE == 2) {
        // lane 0 (c = 0) owns the slice's longest chunk, so it is active at every step
        const uint64_t m = __ballot(changed);
        if (lane == 0) {
          pend.m = m;
          pend.mi = (off + (int64_t)s * S) / S;
        }
      }
    }
  }
  if constexpr (!INIT) {
    pend.flush(a, KS);
    if (a.chg_count) add_wave_count(a.chg_count, nchg);
  }
  sweep_epilogue<G, KP>(a, red, doc, live, chunk, kbase, n, INIT);
}

// #{j : excl + P_j ≤ thr} over a lane's monotone prefix P (branch-free binary search; exact
// because fl(excl + x) is monotone in x). Shared by k_gibbs_x1 (excl = 0) and k_gibbs_ldsg.
template <int KP>
__device__ __forceinline__ int count_le(const float (&P)[KP], float excl, float thr) {
  if constexpr (KP == 16) {
    if (excl + P[15] <= thr) return 16;
    const bool b3 = excl + P[7] <= thr;
    const bool b2 = excl + (b3 ? P[11] : P[3]) <= thr;
    const float a1 = b2 ? P[5] : P[1], a2 = b2 ? P[13] : P[9];
    const bool b1 = excl + (b3 ? a2 : a1) <= thr;
    const float c0 = b1 ? P[2] : P[0], c1 = b1 ? P[6] : P[4], c2 = b1 ? P[10] : P[8], c3 = b1 ? P[14] : P[12];
    const float d0 = b2 ? c1 : c0, d1 = b2 ? c3 : c2;
    const bool b0 = excl + (b3 ? d1 : d0) <= thr;
    return (b3 ? 8 : 0) + (b2 ? 4 : 0) + (b1 ? 2 : 0) + (b0 ? 1 : 0);
  } else if constexpr (KP == 8) {
    if (excl + P[7] <= thr) return 8;
    const bool b2 = excl + P[3] <= thr;
    const bool b1 = excl + (b2 ? P[5] : P[1]) <= thr;
    const float c0 = b1 ? P[2] : P[0], c1 = b1 ? P[6] : P[4];
    const bool b0 = excl + (b2 ? c1 : c0) <= thr;
    return (b2 ? 4 : 0) + (b1 ? 2 : 0) + (b0 ? 1 : 0);
  } else if constexpr (KP > 16 && KP <= 32) {
    // upper or lower 16 by one compare, then the 16-wide search over the selected half (entries
    // past KP read +inf: never counted, thr is finite)
    const bool hi = excl + P[15] <= thr;
    float Q[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) Q[j] = hi ? (16 + j < KP ? P[(16 + j) % KP] : __builtin_inff()) : P[j];
    return (hi ? 16 : 0) + count_le<16>(Q, excl, thr);
  } else if constexpr (KP > 8 && KP < 16) {
    const bool hi = excl + P[7] <= thr;
    float Q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) Q[j] = hi ? (8 + j < KP ? P[(8 + j) % KP] : __builtin_inff()) : P[j];
    return (hi ? 8 : 0) + count_le<8>(Q, excl, thr);
  } else {
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < KP; ++j) cnt += (excl + P[j] <= thr);
    return cnt;
  }
}

// ---- one-lane sweep kernel (K ≤ 32): k_gibbs_x1 ----------------------------------------------------
// Per token and topic slot j the loop body is
//   * 3 ops of count update: the row r_j = n_dj + α is f32 (exact: the host checks, `flags`
//     bit 0) and ONE fused update per step applies +1 at the previous token's new topic and −1 at
//     this token's old topic (the doc-side exclusion) from a 2-bit-field mask M:
//     r_j += (float)bfe_i32(M, 2j, 2) -- no per-slot compare / select chains on the row;
//   * compare + fma + select to put q' = fma(q_j, A, −B) in place of q_zo (no gather of q_{w,zo}:
//     the row is already in registers), 1 fma for the weight chain, compare + add-with-carry count.
// ≈ 240 vector instructions per step at K = 20 (the r3 register sampler: ≈ 380).
// The q row of the next token is fetched a full step ahead into the other register set (static
// roles: the loop is unrolled by two) when its word differs, else copied; token words / topics
// stream two steps ahead in parity slots. Measured (profiles/r4/ab_x1_variants_k20.json): loading
// the next row unconditionally (+0.055 ms/sweep: every lane's 80 B row through the TA each step),
// a ballot-bit-plane count on the scalar unit (+0.013 ms), the q_{w,zo} gather (+0.025 ms) and a
// 3-wave register budget (+0.011 ms) all lost.
// WPD (off: measured 0.255 vs 0.248 ms/sweep): MODE 3/4 changed tokens load their word-sorted
// slot when they change (exec-masked, ~10 % of lanes) instead of streaming it with every token.
template <int KP, int MODE, bool AIR, bool WPD, bool ALN = false, bool LAG = false, bool PKQ = false,
          bool LUT = false>
struct X1 {
  static constexpr int KS = KP;
  static constexpr bool WPF = (MODE == 3 || MODE == 4) && !WPD;
  const OniGibbs& a;
  const float2* qfx;  // LDS: (A, B) per topic
  const float2* dlut;  // LUT: LDS, the (Δ_2p, Δ_2p+1) pair of every 4-bit field pair of the mask
  int lane;
  int64_t off;
  int len;
  float r[KP];
  // token stream in parity slots with static roles (the loop is unrolled by two): slot s & 1
  // holds token s, the other slot token s + 1. Shifting one register set into another while its
  // loads are in flight made the loop latch wait for every outstanding memory op (vmcnt(0)).
  uint32_t ws[2];
  int zs[2];
  int32_t ps[2];
  int ls[2];  // LAG: the tokens' topics in the counts behind q (tok_zlag)
  PhiloxPair rng;
  uint32_t pinc_lo, pinc_hi;  // 2-bit field +1 at the previous token's new topic (pending)
  int znp;                    // that topic (-1: none pending)
  int nchg;
  Pend<MODE> pend;

  __device__ __forceinline__ X1(const OniGibbs& a_, const float2* q_) : a(a_), qfx(q_) {}

  __device__ __forceinline__ void add_fields(uint32_t mlo, uint32_t mhi) {
    if constexpr (LUT) {
      // the two 2-bit fields of a topic pair index a 16-entry LDS table of float pairs: one field
      // extract, one ds_read_b64 and one v_pk_add_f32 per pair instead of two bfe + two cvt + an
      // add (ISA: 733 against 789 VALU per two-step loop; 0.2303-0.2328 against 0.2406-0.2432 ms
      // per sweep, profiles/r6/count_lut/)
      using f2 = float __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int p = 0; p < KP / 2; ++p) {
        const uint32_t m = 2 * p < 16 ? mlo : mhi;
        const float2 d = dlut[__builtin_amdgcn_ubfe(m, 4u * (uint32_t)(p & 7), 4u)];
        f2 v = f2{r[2 * p], r[2 * p + 1]} + f2{d.x, d.y};
        r[2 * p] = v.x;
        r[2 * p + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        const uint32_t m = j < 16 ? mlo : mhi;
        const int sh = 30 - 2 * (j & 15);
        r[j] += (float)((int32_t)(m << sh) >> 30);
      }
    }
  }

  template <int PAR, bool LOAD>
  __device__ __forceinline__ void step(int s, const float (&qc)[KP], float (&qn)[KP]) {
    constexpr int NX = 1 - PAR;
    const int64_t idx = off + (int64_t)s * 64 + lane;
    const uint32_t w = ws[PAR];
    const int zo = zs[PAR];
    const int zl = LAG ? ls[PAR] : zo;
    const int32_t pw = ps[PAR];
    // token s+1: its q row into the other register set (copied when the word repeats)
    if (ws[NX] != oni::kPadWord) {
      if (ws[NX] != w) {
        load_row_f<KP>(a.q + (int64_t)ws[NX] * KS, qn);
      } else {
#pragma unroll
        for (int j = 0; j < KP; ++j) qn[j] = qc[j];
      }
    }
    // token s+2 into this step's slot (LOAD: s + 2 < len, known statically in the main loop)
    if constexpr (LOAD) {
      ws[PAR] = a.tok_word[idx + 128];
      zs[PAR] = (int)a.tok_z[idx + 128];
      if constexpr (LAG) ls[PAR] = (int)a.tok_zlag[idx + 128];
      if constexpr (WPF) ps[PAR] = a.wpos[idx + 128];
    } else {
      ws[PAR] = oni::kPadWord;
    }
    pend.flush(a, KS);
    rng.step(s, a);
    if (w == oni::kPadWord) return;
    const uint32_t rr = ALN ? rng.pick_aligned(s) : rng.pick(s);
    // fused count update: +1 at the previous token's new topic, −1 at this token's old topic
    {
      const uint32_t sh = 2u * (uint32_t)zo;
      uint32_t dlo = sh < 32u ? (3u << sh) : 0u;
      uint32_t dhi = sh >= 32u ? (3u << (sh - 32u)) : 0u;
      uint32_t mlo = pinc_lo | dlo, mhi = pinc_hi | dhi;
      if (znp == zo) mlo = mhi = 0u;
      add_fields(mlo, mhi);
    }
    const float2 ab = qfx[zl];
    float P[KP];
    float run = 0.f;
    if constexpr (PKQ) {
      // q' = fma(q_j, A, −B) on topic pairs (v_pk_fma_f32) inside the chain, so only the pair in
      // flight is live (materialising all KP q' values first spilled at the 4-wave budget)
      using f2 = float __attribute__((ext_vector_type(2)));
      const f2 A2 = {ab.x, ab.x}, B2 = {-ab.y, -ab.y};
#pragma unroll
      for (int j = 0; j < KP; j += 2) {
        const f2 e = __builtin_elementwise_fma(f2{qc[j], qc[j + 1]}, A2, B2);
        run = fmaf(AIR ? r[j] : r[j] + a.alpha, j == zl ? e.x : qc[j], run);
        P[j] = run;
        run = fmaf(AIR ? r[j + 1] : r[j + 1] + a.alpha, j + 1 == zl ? e.y : qc[j + 1], run);
        P[j + 1] = run;
      }
    } else {
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        const float qj = j == zl ? fmaf(qc[j], ab.x, -ab.y) : qc[j];
        run = fmaf(AIR ? r[j] : r[j] + a.alpha, qj, run);
        P[j] = run;
      }
    }
    const float thr = oni::u01(rr) * run;
    int cnt = 0;
    if constexpr (KP > 16) {
      // the first 16 slots by a binary search over the monotone prefix (~20 VALU instead of 32),
      // the rest linearly: the same count
      float P16[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) P16[j] = P[j];
      cnt = count_le<16>(P16, 0.f, thr);
#pragma unroll
      for (int j = 16; j < KP; ++j) cnt += (P[j] <= thr);
    } else {
#pragma unroll
      for (int j = 0; j < KP; ++j) cnt += (P[j] <= thr);
    }
    const int zn = cnt < a.K - 1 ? cnt : a.K - 1;
    {
      const uint32_t sh = 2u * (uint32_t)zn;
      pinc_lo = sh < 32u ? (1u << sh) : 0u;
      pinc_hi = sh >= 32u ? (1u << (sh - 32u)) : 0u;
      znp = zn;
    }
    if constexpr (LAG) {
      if (zl != zo) a.tok_zlag[idx] = (uint8_t)zo;
    }
    const bool changed = zn != zo;
    if (changed) {
      ++nchg;
      int32_t p = pw;
      if constexpr (WPD && (MODE == 3 || MODE == 4)) p = a.wpos[idx];  // used by the next step's flush
      pend.note(idx, zo, zn, p, w);
    }
    if constexpr (MODE == 2) {
      const uint64_t m = __ballot(changed);
      if (lane == 0) {
        pend.m = m;
        pend.mi = (off + (int64_t)s * 64) / 64;
      }
    }
  }
};

// 4 waves per SIMD up to KP = 24 (≤ 128 VGPRs: 3 rows of KP plus the weights); wider rows take
// what they need (a forced 4-wave budget spills at KP = 32)
// LAG streams one more topic per token: 3 waves per SIMD (≤ 168 VGPRs) -- at the 4-wave budget it spilled
template <int KP, int MODE, bool AIR, bool WPD = false, bool ALN = false, bool LAG = false, bool PKQ = false,
          bool LUT = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KP <= 24 ? (LAG ? 3 : 4) : 1, 8))) void k_gibbs_x1(
    const OniGibbs a) {
  static_assert(KP <= 32 && KP % 4 == 0, "one-lane units hold at most 32 topics");
  if (a.exact_guard != nullptr && *a.exact_guard == 0) return;  // a count may leave f32 exactness: generic
  __shared__ float2 qfx[KP];
  __shared__ float2 dlut[16];
  __shared__ int32_t red[kWavesPerBlock][KP];
  if (threadIdx.x < KP) qfx[threadIdx.x] = make_float2(a.qfix[threadIdx.x], a.qfix[KP + threadIdx.x]);
  if (LUT && threadIdx.x < 16) {
    const int lo = (int)(threadIdx.x & 3u), hi = (int)(threadIdx.x >> 2);  // 2-bit fields: 0, +1, (−2), −1
    dlut[threadIdx.x] = make_float2((float)((lo << 30) >> 30), (float)((hi << 30) >> 30));
  }
  __syncthreads();

  using XT = X1<KP, MODE, AIR, WPD, ALN, LAG, PKQ, LUT>;
  XT x(a, qfx);
  x.dlut = dlut;
  const int wave = threadIdx.x >> 6;
  x.lane = threadIdx.x & 63;
  const int64_t slice = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const bool valid = slice < a.n_slices;
  const int64_t chunk = slice * 64 + x.lane;
  const int doc = valid ? a.chunk_doc[chunk] : -1;
  const bool live = doc >= 0;
  {
    int32_t n0[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) n0[j] = 0;
    if (live) load_row_i<KP>(a.ndk_src + (int64_t)doc * KP, n0);
#pragma unroll
    for (int j = 0; j < KP; ++j) x.r[j] = AIR ? (float)n0[j] + a.alpha : (float)n0[j];
  }
  x.len = valid ? a.slice_len[slice] : 0;
  x.off = valid ? a.slice_off[slice] : 0;
  const uint32_t key = live ? a.chunk_key[chunk] : 0u;
  const uint32_t pos0 = live ? (uint32_t)a.chunk_pos0[chunk] : 0u;
  x.rng.init(pos0, key, *a.sweep_ctr, 1u, a);
  x.pinc_lo = x.pinc_hi = 0u;
  x.znp = -1;
  x.nchg = 0;
  const int len = x.len;
  const int64_t off = x.off;
  const int c = x.lane;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    x.ws[t] = len > t ? a.tok_word[off + t * 64 + c] : oni::kPadWord;
    x.zs[t] = len > t ? (int)a.tok_z[off + t * 64 + c] : 0;
    x.ls[t] = (LAG && len > t) ? (int)a.tok_zlag[off + t * 64 + c] : 0;
    x.ps[t] = (XT::WPF && len > t) ? a.wpos[off + t * 64 + c] : 0;
  }
  float qa[KP], qb[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) qa[j] = qb[j] = 0.f;
  if (x.ws[0] != oni::kPadWord) load_row_f<KP>(a.q + (int64_t)x.ws[0] * KP, qa);
  // main loop: every step's look-ahead load is in range, so no value of the token stream is a
  // merge of a load and a constant (such a merge made the latch wait for all memory ops)
  int s = 0;
  for (; s + 3 < len; s += 2) {
    x.template step<0, true>(s, qa, qb);
    x.template step<1, true>(s + 1, qb, qa);
  }
  for (; s < len; s += 2) {  // the last ≤ 3 steps
    if (s + 2 < len) x.template step<0, true>(s, qa, qb);
    else x.template step<0, false>(s, qa, qb);
    if (s + 1 < len) x.template step<1, false>(s + 1, qb, qa);
  }
  x.pend.flush(a, KP);
  x.add_fields(x.pinc_lo, x.pinc_hi);  // the last token's +1
  if (a.chg_count) add_wave_count(a.chg_count, x.nchg);
  int32_t n[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) n[j] = (int32_t)(AIR ? x.r[j] - a.alpha : x.r[j]);
  sweep_epilogue<1, KP>(a, red, doc, live, chunk, 0, n, false);
}

// ---- multi-lane units (K > 32) with LDS-staged counts: k_gibbs_ldsg --------------------------------
//  * lane (unit c, g) keeps its KP counts n + α as f32 in a private LDS row (the host guarantees
//    exactness, `flags` bit 0), so each count update is one LDS read-modify-write by the owner;
//  * the weights form an fma chain P_j = fma(e_j, q_j, P_{j-1}) inside the lane followed by a DPP
//    Hillis-Steele scan across the unit; the token exclusion scales the owner lane's row entry of
//    zo by f = q'/q_zo for the one step (e_zo = a_zo · f), the q row stays in registers;
//  * the count #{j : excl + P_j ≤ thr} is a branch-free binary search over the lane's monotone
//    prefix -- exact because fl(excl + x) is monotone in x.
// Row stride is an odd number of 16-B slots → conflict-free ds_read_b128.
template <int KP>
struct LdsRow {
  static constexpr int kSlots = ((KP / 4) % 2 == 0) ? KP / 4 + 1 : KP / 4;
};

// Sum of an int over each aligned group of G ∈ {2, 4, 8, 16} lanes with DPP butterflies.
template <int G>
__device__ __forceinline__ int group_sum_dpp(int v) {
  static_assert(G == 2 || G == 4 || G == 8 || G == 16, "DPP group sums need G in {2, 4, 8, 16}");
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
  if constexpr (G >= 4) v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
  if constexpr (G >= 8) v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, true);  // row_half_mirror
  if constexpr (G >= 16) v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, true);  // row_mirror
  return v;
}

// Float Hillis-Steele inclusive scan over aligned groups of G ≤ 16 lanes with DPP row shifts: the
// same additions in the same order as the __shfl_up scan of k_gibbs (bitwise identical).
template <int D>
__device__ __forceinline__ float dpp_row_shr(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x110 + D, 0xF, 0xF, true));
}

template <int G>
__device__ __forceinline__ float group_scan_dpp(float x, int g) {
  static_assert(G == 2 || G == 4 || G == 8 || G == 16, "DPP group scans need G in {2, 4, 8, 16}");
  float y = dpp_row_shr<1>(x);
  if (g >= 1) x = x + y;
  if constexpr (G >= 4) {
    y = dpp_row_shr<2>(x);
    if (g >= 2) x = x + y;
  }
  if constexpr (G >= 8) {
    y = dpp_row_shr<4>(x);
    if (g >= 4) x = x + y;
  }
  if constexpr (G >= 16) {
    y = dpp_row_shr<8>(x);
    if (g >= 8) x = x + y;
  }
  return x;
}

// Per-step state of k_gibbs_ldsg. As in k_gibbs_x1 the q rows of consecutive tokens ping-pong
// between two register sets with static roles (loop unrolled by two): the next token's row and its
// own-topic value q_{w,zo} are issued a full step before they are used, so neither the word-change
// row fetch nor the exclusion's gather is a dependent round trip inside the step.
// The Philox word of token s for an aligned unit (every chunk starts at a multiple of 4 tokens):
// its word index s & 3 and the lane of the unit holding its block, (s >> 2) − (s_ref >> 2), are
// both wave-uniform, so the pick is a scalar choice and the exchange one DPP quad permute
// instead of a ds_bpermute (G ∈ {2, 4}: a unit lies inside one quad).
template <int G>
__device__ __forceinline__ uint32_t unit_word(const oni::U4& r, int s, int off) {
  int v;
  switch (s & 3) {
    case 0: v = (int)r.x; break;
    case 1: v = (int)r.y; break;
    case 2: v = (int)r.z; break;
    default: v = (int)r.w; break;
  }
  if constexpr (G == 2) {
    return (uint32_t)(off == 0 ? __builtin_amdgcn_update_dpp(0, v, 0xA0, 0xF, 0xF, false)    // [0,0,2,2]
                               : __builtin_amdgcn_update_dpp(0, v, 0xF5, 0xF, 0xF, false));  // [1,1,3,3]
  } else {
    switch (off) {
      case 0: return (uint32_t)__builtin_amdgcn_update_dpp(0, v, 0x00, 0xF, 0xF, false);
      case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, v, 0x55, 0xF, 0xF, false);
      case 2: return (uint32_t)__builtin_amdgcn_update_dpp(0, v, 0xAA, 0xF, 0xF, false);
      default: return (uint32_t)__builtin_amdgcn_update_dpp(0, v, 0xFF, 0xF, 0xF, false);
    }
  }
}

template <int G, int KP, int MODE, bool ALN = false, bool LAG = false>
struct LG {
  static constexpr int S = oni::kWave / G;
  static constexpr int KS = G * KP;
  static constexpr int kRefresh = 4 * G - 3;
  static constexpr bool WPF = MODE == 3 || MODE == 4;
  const OniGibbs& a;
  const float2* qfx;
  float4* row;
  int lane, c, g, kbase;
  int64_t off;
  int len;
  uint32_t ws[2];  // parity slots with static roles, as in X1
  int zs[2];
  int32_t ps[2];
  int ls[2];  // LAG: the tokens' topics in the counts behind q (tok_zlag)
  float qzs[2];
  uint32_t pos0, key, sweep, gbase;
  oni::U4 r;
  int next_refresh;
  int nchg;
  Pend<MODE> pend;

  __device__ __forceinline__ LG(const OniGibbs& a_, const float2* q_) : a(a_), qfx(q_) {}

  template <int PAR, bool LOAD>
  __device__ __forceinline__ void step(int s, const float (&qc)[KP], float (&qn)[KP]) {
    constexpr int NX = 1 - PAR;
    float* rowf = reinterpret_cast<float*>(row);
    const int64_t idx = off + (int64_t)s * S + c;
    const uint32_t w = ws[PAR];
    const int zo = zs[PAR];
    const int zl = LAG ? ls[PAR] : zo;
    const int32_t pw = ps[PAR];
    const float qz = qzs[PAR];
    if (ws[NX] != oni::kPadWord) {
      const float* qr = a.q + (int64_t)ws[NX] * KS;
      load_row_f<KP>(qr + kbase, qn);
      qzs[NX] = qr[LAG ? ls[NX] : zs[NX]];
    }
    if constexpr (LOAD) {
      ws[PAR] = a.tok_word[idx + 2 * S];
      zs[PAR] = (int)a.tok_z[idx + 2 * S];
      if constexpr (LAG) ls[PAR] = (int)a.tok_zlag[idx + 2 * S];
      if constexpr (WPF) ps[PAR] = a.wpos[idx + 2 * S];
    } else {
      ws[PAR] = oni::kPadWord;
    }
    pend.flush(a, KS);  // after this step's loads
    if (s == next_refresh) {  // wave-uniform (before the pad test: every lane takes it together)
      next_refresh += kRefresh;
      gbase = (pos0 + (uint32_t)s) >> 2;
      r = oni::philox10(oni::U4{gbase + (uint32_t)g, key, sweep, 1u}, a.seed0, a.seed1);
    }
    if (w == oni::kPadWord) return;  // uniform across the G lanes of a unit
    uint32_t rr;
    if constexpr (ALN && (G == 2 || G == 4)) {
      rr = unit_word<G>(r, s, (s >> 2) - ((next_refresh - kRefresh) >> 2));
    } else {
      const uint32_t pos = pos0 + (uint32_t)s;
      const uint32_t gi = pos >> 2;
      rr = (uint32_t)__shfl((int)oni::pick4(r, pos & 3u), (int)(gi - gbase), G);
    }
    const unsigned zlo = (unsigned)(zo - kbase);
    const unsigned zll = LAG ? (unsigned)(zl - kbase) : zlo;
    const float2 ab = qfx[zl];
    const float qe = fmaf(qz, ab.x, -ab.y);
    const float f = qe / qz;
    float tz = 0.f;
    if constexpr (LAG) {
      if (zlo < (unsigned)KP) rowf[zlo] -= 1.0f;  // n^¬t + α (doc side, at the sweep-start topic)
      if (zll < (unsigned)KP) {
        tz = rowf[zll];
        rowf[zll] = tz * f;    // e_zl for this step only (word-side exclusion at the lagged topic)
      }
    } else if (zlo < (unsigned)KP) {
      tz = rowf[zlo] - 1.0f;   // n^¬t + α
      rowf[zlo] = tz * f;      // e_zo for this step only
    }
    float P[KP];
    float run = 0.f;
#pragma unroll
    for (int j = 0; j < KP / 4; ++j) {
      const float4 av = row[j];
      run = fmaf(av.x, qc[4 * j + 0], run);
      P[4 * j + 0] = run;
      run = fmaf(av.y, qc[4 * j + 1], run);
      P[4 * j + 1] = run;
      run = fmaf(av.z, qc[4 * j + 2], run);
      P[4 * j + 2] = run;
      run = fmaf(av.w, qc[4 * j + 3], run);
      P[4 * j + 3] = run;
    }
    if (zll < (unsigned)KP) rowf[zll] = tz;
    const float incl = group_scan_dpp<G>(run, g);
    float excl = dpp_row_shr<1>(incl);
    if (g == 0) excl = 0.f;
    const float total = __shfl(incl, G - 1, G);
    const float thr = oni::u01(rr) * total;
    const int cnt = group_sum_dpp<G>(count_le<KP>(P, excl, thr));
    const int zn = cnt < a.K - 1 ? cnt : a.K - 1;
    const unsigned znl = (unsigned)(zn - kbase);
    if (znl < (unsigned)KP) rowf[znl] += 1.0f;
    const bool changed = zn != zo && g == 0;
    if (changed) {
      ++nchg;
      pend.note(idx, zo, zn, pw, w);
    }
    if constexpr (LAG) {
      if (g == 0 && zl != zo) a.tok_zlag[idx] = (uint8_t)zo;
    }
    if constexpr (MODE == 2) {
      const uint64_t m = __ballot(changed);
      if (lane == 0) {
        pend.m = m;
        pend.mi = (off + (int64_t)s * S) / S;
      }
    }
  }
};

template <int G, int KP, int MODE, int OCC = 1, bool ALN = false, bool LAG = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void k_gibbs_ldsg(const OniGibbs a) {
  static_assert(G > 1, "G = 1 uses k_gibbs_x1");
  if (a.exact_guard != nullptr && *a.exact_guard == 0) return;  // a count may leave f32 exactness: generic
  constexpr int S = oni::kWave / G;
  constexpr int KS = G * KP;
  constexpr int kSlots = LdsRow<KP>::kSlots;
  __shared__ float4 sa[kBlock * kSlots];
  __shared__ int32_t red[kWavesPerBlock][KS];
  __shared__ float2 qfx[KS];
  for (int k = threadIdx.x; k < KS; k += kBlock) qfx[k] = make_float2(a.qfix[k], a.qfix[KS + k]);
  LG<G, KP, MODE, ALN, LAG> x(a, qfx);
  const int wave = threadIdx.x >> 6;
  x.lane = threadIdx.x & 63;
  x.c = x.lane / G;
  x.g = x.lane % G;
  const int c = x.c, g = x.g;
  const int64_t slice = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const bool valid = slice < a.n_slices;
  const int64_t chunk = slice * S + c;
  const int doc = valid ? a.chunk_doc[chunk] : -1;
  const bool live = doc >= 0;
  x.kbase = g * KP;
  const int kbase = x.kbase;
  x.row = sa + threadIdx.x * kSlots;
  {
    int32_t n0[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) n0[j] = 0;
    if (live) load_row_i<KP>(a.ndk_src + (int64_t)doc * KS + kbase, n0);
#pragma unroll
    for (int j = 0; j < KP / 4; ++j)
      x.row[j] = make_float4((float)n0[4 * j] + a.alpha, (float)n0[4 * j + 1] + a.alpha,
                             (float)n0[4 * j + 2] + a.alpha, (float)n0[4 * j + 3] + a.alpha);
  }
  __syncthreads();  // qfx
  x.len = valid ? a.slice_len[slice] : 0;
  x.off = valid ? a.slice_off[slice] : 0;
  const int len = x.len;
  const int64_t off = x.off;
  x.key = live ? a.chunk_key[chunk] : 0u;
  x.pos0 = live ? (uint32_t)a.chunk_pos0[chunk] : 0u;
  x.sweep = *a.sweep_ctr;
  // Philox blocks are shared by the unit: lane g holds the block of 4-token group gbase + g, so
  // the unit computes one block per G·4 tokens; the refresh is wave-uniform: every
  // kRefresh = 4G - 3 steps each unit recomputes the G blocks that cover its next kRefresh tokens.
  x.gbase = x.pos0 >> 2;
  x.r = oni::philox10(oni::U4{x.gbase + (uint32_t)g, x.key, x.sweep, 1u}, a.seed0, a.seed1);
  x.next_refresh = LG<G, KP, MODE, ALN, LAG>::kRefresh;
  x.nchg = 0;
  constexpr bool WPF = LG<G, KP, MODE, ALN, LAG>::WPF;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    x.ws[t] = len > t ? a.tok_word[off + t * S + c] : oni::kPadWord;
    x.zs[t] = len > t ? (int)a.tok_z[off + t * S + c] : 0;
    x.ps[t] = (WPF && len > t) ? a.wpos[off + t * S + c] : 0;
    x.ls[t] = (LAG && len > t) ? (int)a.tok_zlag[off + t * S + c] : 0;
    x.qzs[t] = 0.f;
  }
  float qa[KP], qb[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) qa[j] = qb[j] = 0.f;
  if (x.ws[0] != oni::kPadWord) {
    const float* qr = a.q + (int64_t)x.ws[0] * KS;
    load_row_f<KP>(qr + kbase, qa);
    x.qzs[0] = qr[LAG ? x.ls[0] : x.zs[0]];
  }
  int s = 0;
  for (; s + 3 < len; s += 2) {
    x.template step<0, true>(s, qa, qb);
    x.template step<1, true>(s + 1, qb, qa);
  }
  for (; s < len; s += 2) {  // the last ≤ 3 steps
    if (s + 2 < len) x.template step<0, true>(s, qa, qb);
    else x.template step<0, false>(s, qa, qb);
    if (s + 1 < len) x.template step<1, false>(s + 1, qb, qa);
  }
  x.pend.flush(a, KS);
  if (a.chg_count) add_wave_count(a.chg_count, x.nchg);
  const float* rowf = reinterpret_cast<const float*>(x.row);
  int32_t n[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) n[j] = (int32_t)(rowf[j] - a.alpha);
  sweep_epilogue<G, KP>(a, red, doc, live, chunk, kbase, n, false);
}

// Sampler variants (the `qpf` launch argument, oni355.models.gibbs SAMPLERS):
//   0 = generic k_gibbs (any G; the fallback), 2 = k_gibbs_ldsg (G > 1), 3 = k_gibbs_x1 (G = 1).
// The specialised kernels need n + α exact in f32 (flags bit 0); otherwise the generic one runs.
template <int G, int KP>
int launch_gibbs_one(const OniGibbs& a, bool init, int mode, int qpf, hipStream_t s);

// With a device exactness guard (a.exact_guard) the row-f32 kernel and the generic kernel are both
// launched; each reads the flag and all but one return at once -- a per-sweep choice that graph
// replays keep making on the device (the same draws either way: every variant replays the oracle).
template <int G, int KP>
int launch_gibbs(const OniGibbs& a, bool init, int mode, int qpf, hipStream_t s) {
  const int rc = launch_gibbs_one<G, KP>(a, init, mode, qpf, s);
  if (rc != 0 || init || a.exact_guard == nullptr || !(a.flags & 1) || (qpf != 2 && qpf != 3)) return rc;
  OniGibbs b = a;
  b.flags = (b.flags & ~1) | 64;  // no row-f32 kernel: the generic one, guarded
  return launch_gibbs_one<G, KP>(b, init, mode, 0, s);
}

template <int G, int KP>
int launch_gibbs_one(const OniGibbs& a, bool init, int mode, int qpf, hipStream_t s) {
  if (a.KS != G * KP || mode < 0 || mode > 4) return (int)hipErrorInvalidValue;
  const unsigned grid = (unsigned)((a.n_slices + kWavesPerBlock - 1) / kWavesPerBlock);
  if (grid == 0) return 0;
  if (init) {
    // mode 1: n_wk by per-token atomics; mode 0: no n_wk bookkeeping, the caller rebuilds it with
    // the word-sorted recount
    if (mode == 0) k_gibbs<G, KP, true, 0><<<grid, kBlock, 0, s>>>(a);
    else k_gibbs<G, KP, true, 1><<<grid, kBlock, 0, s>>>(a);
    return (int)hipGetLastError();
  }
  if (a.qfix == nullptr) return (int)hipErrorInvalidValue;
  const bool air = (a.flags & 1) != 0;
  if (a.tok_zlag != nullptr) {
    // lagged word side: the specialised kernels on the default paths (aligned chunks, recount /
    // wdelta), the generic kernel (which reads tok_zlag at run time) for anything else
    if constexpr (G == 1) {
      if (qpf == 3 && KP <= 32 && air && (a.flags & 16) && !(a.flags & 2) && (mode == 0 || mode == 4)) {
        if (mode == 0) k_gibbs_x1<KP, 0, true, false, true, true><<<grid, kBlock, 0, s>>>(a);
        else k_gibbs_x1<KP, 4, true, false, true, true><<<grid, kBlock, 0, s>>>(a);
        return (int)hipGetLastError();
      }
    } else {
      if (qpf == 2 && air && (a.flags & 16) && (G == 2 || G == 4) && (mode == 0 || mode == 4)) {
        if (mode == 0) k_gibbs_ldsg<G, KP, 0, 1, true, true><<<grid, kBlock, 0, s>>>(a);
        else k_gibbs_ldsg<G, KP, 4, 1, true, true><<<grid, kBlock, 0, s>>>(a);
        return (int)hipGetLastError();
      }
      if (qpf == 2 && air && (mode == 0 || mode == 4)) {
        if (mode == 0) k_gibbs_ldsg<G, KP, 0, 1, false, true><<<grid, kBlock, 0, s>>>(a);
        else k_gibbs_ldsg<G, KP, 4, 1, false, true><<<grid, kBlock, 0, s>>>(a);
        return (int)hipGetLastError();
      }
    }
  } else if constexpr (G == 1) {
    if (qpf == 3 && KP <= 32 && air && (a.flags & 16) && !(a.flags & 2) && (mode == 0 || mode == 4)) {
      // every chunk starts at a multiple of 4 tokens (the default day's path: recount / wdelta);
      // flags bit 5 (ONI_SAMPLER_AB & 4): A/B of the packed q' (v_pk_fma_f32) against the scalar
      // one -- 30 fewer VALU per two steps, 3.5 % slower per sweep (profiles/r6/packed_fp32/)
      if (a.flags & 32) {
        if (mode == 0) k_gibbs_x1<KP, 0, true, false, true, false, true><<<grid, kBlock, 0, s>>>(a);
        else k_gibbs_x1<KP, 4, true, false, true, false, true><<<grid, kBlock, 0, s>>>(a);
        return (int)hipGetLastError();
      }
      if (a.flags & 128) {  // A/B (ONI_SAMPLER_AB & 8): the ±1 count update by per-topic bfe + cvt (round 5)
        if (mode == 0) k_gibbs_x1<KP, 0, true, false, true><<<grid, kBlock, 0, s>>>(a);
        else k_gibbs_x1<KP, 4, true, false, true><<<grid, kBlock, 0, s>>>(a);
        return (int)hipGetLastError();
      }
      // default: the ±1 count update through the LDS table of float pairs (4 % faster per sweep,
      // profiles/r6/count_lut/)
      if (mode == 0) k_gibbs_x1<KP, 0, true, false, true, false, false, true><<<grid, kBlock, 0, s>>>(a);
      else k_gibbs_x1<KP, 4, true, false, true, false, false, true><<<grid, kBlock, 0, s>>>(a);
      return (int)hipGetLastError();
    }
    if (qpf == 3 && KP <= 32) {
      if ((a.flags & 2) && (mode == 3 || mode == 4)) {  // A/B: word-sorted slots loaded on change
        if (air && mode == 4) k_gibbs_x1<KP, 4, true, true><<<grid, kBlock, 0, s>>>(a);
        else if (air) k_gibbs_x1<KP, 3, true, true><<<grid, kBlock, 0, s>>>(a);
        else if (mode == 4) k_gibbs_x1<KP, 4, false, true><<<grid, kBlock, 0, s>>>(a);
        else k_gibbs_x1<KP, 3, false, true><<<grid, kBlock, 0, s>>>(a);
        return (int)hipGetLastError();
      }
      if (air) {
        switch (mode) {
          case 0: k_gibbs_x1<KP, 0, true><<<grid, kBlock, 0, s>>>(a); break;
          case 1: k_gibbs_x1<KP, 1, true><<<grid, kBlock, 0, s>>>(a); break;
          case 2: k_gibbs_x1<KP, 2, true><<<grid, kBlock, 0, s>>>(a); break;
          case 3: k_gibbs_x1<KP, 3, true><<<grid, kBlock, 0, s>>>(a); break;
          default: k_gibbs_x1<KP, 4, true><<<grid, kBlock, 0, s>>>(a); break;
        }
      } else {
        switch (mode) {
          case 0: k_gibbs_x1<KP, 0, false><<<grid, kBlock, 0, s>>>(a); break;
          case 1: k_gibbs_x1<KP, 1, false><<<grid, kBlock, 0, s>>>(a); break;
          case 2: k_gibbs_x1<KP, 2, false><<<grid, kBlock, 0, s>>>(a); break;
          case 3: k_gibbs_x1<KP, 3, false><<<grid, kBlock, 0, s>>>(a); break;
          default: k_gibbs_x1<KP, 4, false><<<grid, kBlock, 0, s>>>(a); break;
        }
      }
      return (int)hipGetLastError();
    }
  } else {
    if (qpf == 2 && air && (a.flags & 4) && (mode == 0 || mode == 4)) {  // A/B: 4-wave register budget
      if (mode == 0) k_gibbs_ldsg<G, KP, 0, 4><<<grid, kBlock, 0, s>>>(a);
      else k_gibbs_ldsg<G, KP, 4, 4><<<grid, kBlock, 0, s>>>(a);
      return (int)hipGetLastError();
    }
    if (qpf == 2 && air && (a.flags & 16) && (G == 2 || G == 4) && (mode == 0 || mode == 4)) {
      // every chunk starts at a multiple of 4 tokens: uniform Philox word, DPP exchange
      if (mode == 0) k_gibbs_ldsg<G, KP, 0, 1, true><<<grid, kBlock, 0, s>>>(a);
      else k_gibbs_ldsg<G, KP, 4, 1, true><<<grid, kBlock, 0, s>>>(a);
      return (int)hipGetLastError();
    }
    if (qpf == 2 && air) {
      switch (mode) {
        case 0: k_gibbs_ldsg<G, KP, 0><<<grid, kBlock, 0, s>>>(a); break;
        case 1: k_gibbs_ldsg<G, KP, 1><<<grid, kBlock, 0, s>>>(a); break;
        case 2: k_gibbs_ldsg<G, KP, 2><<<grid, kBlock, 0, s>>>(a); break;
        case 3: k_gibbs_ldsg<G, KP, 3><<<grid, kBlock, 0, s>>>(a); break;
        default: k_gibbs_ldsg<G, KP, 4><<<grid, kBlock, 0, s>>>(a); break;
      }
      return (int)hipGetLastError();
    }
  }
  switch (mode) {
    case 0: k_gibbs<G, KP, false, 0><<<grid, kBlock, 0, s>>>(a); break;
    case 1: k_gibbs<G, KP, false, 1><<<grid, kBlock, 0, s>>>(a); break;
    case 2: k_gibbs<G, KP, false, 2><<<grid, kBlock, 0, s>>>(a); break;
    case 3: k_gibbs<G, KP, false, 3><<<grid, kBlock, 0, s>>>(a); break;
    default: k_gibbs<G, KP, false, 4><<<grid, kBlock, 0, s>>>(a); break;
  }
  return (int)hipGetLastError();
}

}  // namespace

// Per-unit-width dispatchers (gibbs_g1.hip, gibbs_g2.hip, gibbs_g4.hip, gibbs_g8.hip): launch
// launch_gibbs<G, KP> for a supported KP; hipErrorInvalidValue otherwise.
int oni_gibbs_dispatch_g1(const OniGibbs& a, int KP, bool init, int mode, int qpf, hipStream_t s);
int oni_gibbs_dispatch_g2(const OniGibbs& a, int KP, bool init, int mode, int qpf, hipStream_t s);
int oni_gibbs_dispatch_g4(const OniGibbs& a, int KP, bool init, int mode, int qpf, hipStream_t s);
int oni_gibbs_dispatch_g8(const OniGibbs& a, int G, int KP, bool init, int mode, int qpf, hipStream_t s);
