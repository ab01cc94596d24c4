// Collapsed-Gibbs sweep kernels (K10) and their launcher template, shared by gibbs.hip and the
// per-unit-width instantiation units gibbs_g*.hip (compiled in parallel: one translation unit
// holding every (G, KP) instantiation took ~4 min of a clean build).
#pragma once
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
  int32_t* dnwk;               // [V][KS] word-topic delta (init: the n_wk table itself)
  int32_t* dnk;                // [nk_rep][KS] topic-total delta replicas (init: n_k itself, nk_rep = 1)
  const uint32_t* sweep_ctr;   // device scalar: current sweep number (≥ 1), graph-replay safe
  uint64_t* chg_mask;          // MODE 2: one u64 per SELL step, bit c*G set if slot c's topic changed
  const int32_t* wpos;         // MODE 3: word-sorted position of every SELL slot
  uint8_t* z_w;                // MODE 3: topic array in word-sorted order (kept in sync for changed tokens)
  uint16_t* zz_w;              // MODE 4: (old | new << 8) topics of each changed token, word-sorted order
                               // (MODE 4 reuses chg_mask as a u32 bitmap over word-sorted positions)
  int32_t* chg_count;          // optional: += number of tokens whose topic changed (drives the auto mode)
  int64_t n_slices;
  int32_t K;
  int32_t KS;
  float alpha;
  uint32_t seed0, seed1;
  int32_t nk_rep;              // dnk holds nk_rep replicas of [KS] (power of 2): block b adds into b % nk_rep
  int32_t flags;               // bit 0: LDS samplers may keep n + α in their rows (exact in f32 here)
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
// queue KS × chunks adds on a single row (measured: ~2 ms/sweep in the high-change early sweeps).
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

// MODE 4: a changed token records (old, new) topic at its word-sorted position p and sets bit p
// of a word-sorted bitmap; k_wdelta_recount then visits only set bits, reading contiguous
// word ids and topic pairs (no per-token slot indirection, no z_prev array).
__device__ __forceinline__ void mark_changed_w(const OniGibbs& a, int32_t p, int zo, int zn) {
  a.zz_w[p] = (uint16_t)(zo | (zn << 8));  // one 2-B store: only read where the bit below is set
  atomicOr(reinterpret_cast<uint32_t*>(a.chg_mask) + (p >> 5), 1u << (p & 31));
}

// ---- deferred topic bookkeeping (DZ) ------------------------------------------------------------
// On CDNA every vector-memory operation -- load, store or atomic -- retires through one in-order
// vmcnt counter per wave. A sampler that writes a changed topic (tok_z byte, plus in MODE 4 the
// zz_w pair and the bitmap atomicOr, which stays counted for ~600-3000 cycles) inside its token
// loop therefore makes the NEXT step's wait for its q row also wait for those stores. The DZ
// variant keeps the slice's topics in LDS instead (staged once in the prologue, 64 B per step:
// step s, lane c at byte s·64 + c), so the token loop issues loads only; the epilogue writes the
// slice back with 16-B stores and does the per-mode bookkeeping for the bytes that changed
// (compared against the untouched global copy). Same draws, bit for bit: only where the topic
// lives during the sweep changes. Slices up to kDzMaxLen steps (the auto chunk length is ≤ 128).
constexpr int kDzMaxLen = 128;

template <int MODE>
__device__ __forceinline__ void dz_note_change(const OniGibbs& a, int64_t slot, int zo, int zn) {
  if constexpr (MODE == 1) {
    const int64_t w = (int64_t)a.tok_word[slot];
    atomicAdd(&a.dnwk[w * a.KS + zo], -1);
    atomicAdd(&a.dnwk[w * a.KS + zn], 1);
  } else if constexpr (MODE == 3) {
    a.z_w[a.wpos[slot]] = (uint8_t)zn;
  } else if constexpr (MODE == 4) {
    mark_changed_w(a, a.wpos[slot], zo, zn);
  }
}

// Write a wave's LDS topic stage (len steps × 64 B) back to tok_z and do the MODE bookkeeping of
// every changed byte. Called by all 64 lanes of the wave after a barrier.
template <int MODE>
__device__ __forceinline__ void dz_flush(const OniGibbs& a, const uint32_t* __restrict__ zs, int64_t off, int len,
                                         int lane) {
  const uint4* stage = reinterpret_cast<const uint4*>(zs);
  uint4* dst = reinterpret_cast<uint4*>(a.tok_z + off);
  for (int i = lane; i < len * 4; i += oni::kWave) {
    const uint4 nw = stage[i];
    const uint4 od = dst[i];
    const uint32_t n4[4] = {nw.x, nw.y, nw.z, nw.w}, o4[4] = {od.x, od.y, od.z, od.w};
    bool any = false;
#pragma unroll
    for (int d = 0; d < 4; ++d) any |= n4[d] != o4[d];
    if (!any) continue;
    dst[i] = nw;
    if constexpr (MODE == 1 || MODE == 3 || MODE == 4) {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint32_t x = n4[d] ^ o4[d];
        while (x) {
          const int b = (__ffs(x) - 1) >> 3;
          x &= ~(0xFFu << (8 * b));
          dz_note_change<MODE>(a, off + (int64_t)i * 16 + d * 4 + b, (int)((o4[d] >> (8 * b)) & 0xFFu),
                               (int)((n4[d] >> (8 * b)) & 0xFFu));
        }
      }
    }
  }
}

// Philox blocks at a wave-uniform cadence for samplers with one chain per lane. A lane needs a
// new block whenever its token position enters a new 4-token group; with 64 chunks at random
// phases some lane does so on every step, so the wave issued a whole block (36 quarter-rate
// multiplies) per step for a quarter of its lanes. Here every lane refreshes together every 4
// steps and computes only the block of the group AFTER its current one (within a 4-step window a
// position lies in one of two consecutive groups, and the current group's block is the previous
// refresh's "next"): one block per lane per 4 steps, the same values, the same draws bitwise.
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
  __device__ __forceinline__ uint32_t pick(int s) const {
    const uint32_t pos = pos0 + (uint32_t)s;
    const bool second = (pos >> 2) != ((pos0 + (uint32_t)(s & ~3)) >> 2);
    const uint32_t i = pos & 3u;
    return second ? oni::pick4(nxt, i) : oni::pick4(cur, i);  // value selects: no addressed copy
  }
};

// A changed token's bookkeeping, held back one step (see k_gibbs_ldsg "Deferred bookkeeping").
struct PendZ {
  bool on = false;
  int64_t idx = 0;
  int zo = 0, zn = 0;
  int32_t pw = 0;
  uint32_t w = 0;
  uint64_t m = 0;       // MODE 2: the step's change ballot ...
  uint64_t* mdst = nullptr;  // ... and where lane 0 stores it
};

template <int MODE>
__device__ __forceinline__ void flush_pend(const OniGibbs& a, PendZ& p, int KS) {
  if (p.on) {
    a.tok_z[p.idx] = (uint8_t)p.zn;
    if constexpr (MODE == 3) a.z_w[p.pw] = (uint8_t)p.zn;
    if constexpr (MODE == 4) mark_changed_w(a, p.pw, p.zo, p.zn);
    if constexpr (MODE == 1) {
      atomicAdd(&a.dnwk[(int64_t)p.w * KS + p.zo], -1);
      atomicAdd(&a.dnwk[(int64_t)p.w * KS + p.zn], 1);
    }
    p.on = false;
  }
  if constexpr (MODE == 2) {
    if (p.mdst) *p.mdst = p.m;
    p.mdst = nullptr;
  }
}

// MODE: 0 = no n_wk bookkeeping (full recount afterwards), 1 = per-token Δ atomics,
//       2 = changed-slot ballot mask per step (delta recount afterwards),
//       3 = changed topics also scattered into the word-sorted copy z_w (streaming recount afterwards)
//       4 = changed tokens marked in a word-sorted bitmap + (old, new) topic copies (k_wdelta_recount)
// DZ (G = 1, MODE != 2, not INIT): topics staged in LDS, bookkeeping in the epilogue (see dz_flush).
template <int G, int KP, bool INIT, int MODE, bool QPF, bool DZ = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 4))) void k_gibbs(const OniGibbs a) {
  static_assert(!DZ || (G == 1 && !INIT && MODE != 2), "DZ: one-lane units, sweeps, MODE != 2");
  constexpr bool ATOMIC = MODE == 1 && !DZ;
  constexpr int S = oni::kWave / G;
  constexpr int KS = G * KP;
  __shared__ int32_t red[kWavesPerBlock][KS];
  __shared__ uint32_t zstage[DZ ? kWavesPerBlock : 1][DZ ? kDzMaxLen * 16 : 1];

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
  // QPF: qn always holds the q row of the current token's word (it is refilled at the end of a
  // step only when the next word differs, so a repeated word finds its row still there) and the
  // math reads it directly; without QPF qv holds the row loaded on a word change
  float qv[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) qv[j] = 0.f;

  int nchg = 0;
  uint8_t* zb = DZ ? reinterpret_cast<uint8_t*>(zstage[wave]) : nullptr;
  if constexpr (DZ) {
    // the slice's topics → LDS (slice_off is a multiple of 64 B: 16-B aligned pieces)
    const uint4* src = reinterpret_cast<const uint4*>(a.tok_z + off);
    uint4* stg = reinterpret_cast<uint4*>(zstage[wave]);
    for (int i = lane; i < len * 4; i += oni::kWave) stg[i] = src[i];
    __syncthreads();
  }
  // software-pipelined token stream: step s+1's word/topic loads are issued before step s's
  // sampling, so their latency hides behind the math and stores of step s
  uint32_t w_nx = len > 0 ? a.tok_word[off + c] : oni::kPadWord;
  int z_nx = (!INIT && len > 0) ? (DZ ? (int)zb[c] : (int)a.tok_z[off + c]) : 0;
  // MODE 3/4: the token's word-sorted position streams with its word/topic (a load issued only
  // once the draw is known would expose a full memory latency on almost every step)
  constexpr bool WPF = !INIT && !DZ && (MODE == 3 || MODE == 4);
  int32_t p_nx = (WPF && len > 0) ? a.wpos[off + c] : 0;
  // QPF: the next token's q row is also fetched one step ahead (needs only its word id)
  float qn[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) qn[j] = 0.f;
  if (QPF && !INIT && w_nx != oni::kPadWord) load_row_f<KP>(a.q + (int64_t)w_nx * KS + kbase, qn);
  for (int s = 0; s < len; ++s) {
    const int64_t idx = off + (int64_t)s * S + c;
    const uint32_t w = w_nx;
    const int zo = z_nx;
    const int32_t pw = p_nx;
    if (s + 1 < len) {
      w_nx = a.tok_word[idx + S];
      if (!INIT) z_nx = DZ ? (int)zb[(s + 1) * S + c] : (int)a.tok_z[idx + S];
      if (WPF) p_nx = a.wpos[idx + S];
    }
    rng.step(s, a);
    if (w == oni::kPadWord) continue;  // uniform across the G lanes of a unit
    const uint32_t rr = rng.pick(s);
    if constexpr (INIT) {
      const int z = (int)__umulhi(rr, (uint32_t)a.K);
#pragma unroll
      for (int j = 0; j < KP; ++j) n[j] += (kbase + j == z);
      if (g == 0) {
        a.tok_z[idx] = (uint8_t)z;
        if (ATOMIC) atomicAdd(&a.dnwk[(int64_t)w * KS + z], 1);
      }
    } else {
#pragma unroll
      for (int j = 0; j < KP; ++j) n[j] -= (kbase + j == zo);
      if constexpr (!QPF) {
        if (w != wprev) {
          load_row_f<KP>(a.q + (int64_t)w * KS + kbase, qv);
          wprev = w;
        }
      }
      float loc[KP];
      float run = 0.f;
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        run = run + ((float)n[j] + a.alpha) * (QPF ? qn[j] : qv[j]);
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
      if constexpr (DZ) {
        // LDS only: no vector-memory store in the token loop
        nchg += zn != zo;
        if (zn != zo) zb[s * S + c] = (uint8_t)zn;
      } else if (zn != zo && g == 0) {
        ++nchg;
        a.tok_z[idx] = (uint8_t)zn;
        if constexpr (MODE == 3) a.z_w[pw] = (uint8_t)zn;
        if constexpr (MODE == 4) mark_changed_w(a, pw, zo, zn);
        if (ATOMIC) {
          atomicAdd(&a.dnwk[(int64_t)w * KS + zo], -1);
          atomicAdd(&a.dnwk[(int64_t)w * KS + zn], 1);
        }
      }
      if constexpr (MODE == 2 && !DZ) {
        // lane 0 (c = 0) owns the slice's longest chunk, so it is active at every step
        const uint64_t m = __ballot(zn != zo && g == 0);
        if (lane == 0) a.chg_mask[(off + (int64_t)s * S) / S] = m;
      }
      if (QPF && s + 1 < len && w_nx != w && w_nx != oni::kPadWord)
        load_row_f<KP>(a.q + (int64_t)w_nx * KS + kbase, qn);
    }
  }

  // ---- epilogue: doc rows + per-topic totals -------------------------------------------------
  if (!INIT && a.chg_count) add_wave_count(a.chg_count, nchg);
  if constexpr (DZ) {
    __syncthreads();  // every lane's LDS topic writes before the wave reads the stage back
    dz_flush<MODE>(a, zstage[wave], off, len, lane);
  }
  int32_t d[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) d[j] = 0;
  if (live) {
    int32_t* dst = a.ndk_dst + (int64_t)doc * KS + kbase;
    if (INIT) {
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

// ---- two-deep token stream, q row issued a full step ahead (G = 1) -----------------------------
// k_gibbs<.., QPF = true> fetches the next token's q row at the END of a step and consumes it at
// the top of the next one: with ~11 % of tokens starting a new word, some lane of a wave needs a
// row on almost every step, so that L2 round trip is exposed once per step (the dominant
// s_waitcnt stall in the K = 20 counters). Here token words/topics/slots stream two steps ahead,
// so token s+1's word is already in registers at the top of step s: its q row is issued there,
// before step s's math and stores, and waited for only when the step ends. Same arithmetic as
// k_gibbs (mul + add chain), so the same draws bitwise.
// DZ: the topics live in LDS during the sweep (see dz_flush): the loop issues loads only.
template <int KP, int MODE, bool DZ = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 4))) void k_gibbs_q2(const OniGibbs a) {
  static_assert(!DZ || MODE != 2, "DZ: MODE != 2");
  constexpr bool ATOMIC = MODE == 1 && !DZ;
  constexpr int S = oni::kWave;
  constexpr int KS = KP;
  __shared__ int32_t red[kWavesPerBlock][KS];
  __shared__ uint32_t zstage[DZ ? kWavesPerBlock : 1][DZ ? kDzMaxLen * 16 : 1];

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int c = lane;
  const int64_t slice = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const bool valid = slice < a.n_slices;
  const int64_t chunk = slice * S + c;
  const int doc = valid ? a.chunk_doc[chunk] : -1;
  const bool live = doc >= 0;

  int32_t n[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) n[j] = 0;
  if (live) load_row_i<KP>(a.ndk_src + (int64_t)doc * KS, n);

  const int len = valid ? a.slice_len[slice] : 0;
  const int64_t off = valid ? a.slice_off[slice] : 0;
  const uint32_t key = live ? a.chunk_key[chunk] : 0u;
  const uint32_t pos0 = live ? (uint32_t)a.chunk_pos0[chunk] : 0u;
  const uint32_t sweep = *a.sweep_ctr;

  uint8_t* zb = DZ ? reinterpret_cast<uint8_t*>(zstage[wave]) : nullptr;
  if constexpr (DZ) {
    const uint4* src = reinterpret_cast<const uint4*>(a.tok_z + off);
    uint4* stg = reinterpret_cast<uint4*>(zstage[wave]);
    for (int i = lane; i < len * 4; i += oni::kWave) stg[i] = src[i];
    __syncthreads();
  }
  constexpr bool WPF = !DZ && (MODE == 3 || MODE == 4);
  // token stream: (w0, z0, p0) = token s, (w1, z1, p1) = token s + 1
  uint32_t w0 = len > 0 ? a.tok_word[off + c] : oni::kPadWord;
  int z0 = len > 0 ? (DZ ? (int)zb[c] : (int)a.tok_z[off + c]) : 0;
  int32_t p0 = (WPF && len > 0) ? a.wpos[off + c] : 0;
  uint32_t w1 = len > 1 ? a.tok_word[off + S + c] : oni::kPadWord;
  int z1 = len > 1 ? (DZ ? (int)zb[S + c] : (int)a.tok_z[off + S + c]) : 0;
  int32_t p1 = (WPF && len > 1) ? a.wpos[off + S + c] : 0;
  float qv[KP], qn[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) qv[j] = qn[j] = 0.f;
  if (w0 != oni::kPadWord) load_row_f<KP>(a.q + (int64_t)w0 * KS, qv);

  PhiloxPair rng;
  rng.init(pos0, key, sweep, 1u, a);
  int nchg = 0;
  // deferred bookkeeping (as k_gibbs_ldsg): a changed token's stores are issued in the next step,
  // after its q-row and token-stream loads, so the wait for those loads at the top of the step
  // after does not also wait out the stores (vmcnt retires in issue order)
  bool pend = false;
  int64_t p_idx = 0;
  int p_zo = 0, p_zn = 0;
  int32_t p_pw = 0;
  uint32_t p_w = 0;
  uint64_t p_m = 0;
  int64_t p_mi = -1;
  auto flush = [&]() {
    if constexpr (!DZ) {
      if (pend) {
        a.tok_z[p_idx] = (uint8_t)p_zn;
        if constexpr (MODE == 3) a.z_w[p_pw] = (uint8_t)p_zn;
        if constexpr (MODE == 4) mark_changed_w(a, p_pw, p_zo, p_zn);
        if (ATOMIC) {
          atomicAdd(&a.dnwk[(int64_t)p_w * KS + p_zo], -1);
          atomicAdd(&a.dnwk[(int64_t)p_w * KS + p_zn], 1);
        }
        pend = false;
      }
      if constexpr (MODE == 2) {
        if (p_mi >= 0) a.chg_mask[p_mi] = p_m;
        p_mi = -1;
      }
    }
  };
  for (int s = 0; s < len; ++s) {
    const int64_t idx = off + (int64_t)s * S + c;
    const uint32_t w = w0;
    const int zo = z0;
    const int32_t pw = p0;
    // token s+1's q row now (consumed after this step's math): a full step of latency hiding
    const bool fetch = w1 != oni::kPadWord && w1 != w;
    if (fetch) load_row_f<KP>(a.q + (int64_t)w1 * KS, qn);
    // advance the token stream: token s+2's loads queue behind the q row
    w0 = w1;
    z0 = z1;
    p0 = p1;
    if (s + 2 < len) {
      w1 = a.tok_word[idx + 2 * S];
      z1 = DZ ? (int)zb[(s + 2) * S + c] : (int)a.tok_z[idx + 2 * S];
      if (WPF) p1 = a.wpos[idx + 2 * S];
    } else {
      w1 = oni::kPadWord;
    }
    flush();
    rng.step(s, a);
    if (w != oni::kPadWord) {
      const uint32_t rr = rng.pick(s);
#pragma unroll
      for (int j = 0; j < KP; ++j) n[j] -= (j == zo);
      float loc[KP];
      float run = 0.f;
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        run = run + ((float)n[j] + a.alpha) * qv[j];
        loc[j] = run;
      }
      const float thr = oni::u01(rr) * run;
      int cnt = 0;
#pragma unroll
      for (int j = 0; j < KP; ++j) cnt += (loc[j] <= thr);
      const int zn = cnt < a.K - 1 ? cnt : a.K - 1;
#pragma unroll
      for (int j = 0; j < KP; ++j) n[j] += (j == zn);
      if constexpr (DZ) {
        nchg += zn != zo;
        if (zn != zo) zb[s * S + c] = (uint8_t)zn;
      } else if (zn != zo) {
        ++nchg;
        pend = true;
        p_idx = idx;
        p_zo = zo;
        p_zn = zn;
        p_pw = pw;
        p_w = w;
      }
      if constexpr (MODE == 2 && !DZ) {
        const uint64_t m = __ballot(zn != zo);
        if (lane == 0) {
          p_m = m;
          p_mi = (off + (int64_t)s * S) / S;
        }
      }
    }
    if (fetch) {
#pragma unroll
      for (int j = 0; j < KP; ++j) qv[j] = qn[j];
    }
  }
  flush();

  // ---- epilogue: doc rows + per-topic totals (as k_gibbs, G = 1) --------------------------------
  if (a.chg_count) add_wave_count(a.chg_count, nchg);
  if constexpr (DZ) {
    __syncthreads();
    dz_flush<MODE>(a, zstage[wave], off, len, lane);
  }
  int32_t d[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) d[j] = 0;
  if (live) {
    int32_t* dst = a.ndk_dst + (int64_t)doc * KS;
    int32_t n0[KP];
    load_row_i<KP>(a.ndk_src + (int64_t)doc * KS, n0);
#pragma unroll
    for (int j = 0; j < KP; ++j) d[j] = n[j] - n0[j];
    if (!a.chunk_multi[chunk]) {
#pragma unroll
      for (int j = 0; j < KP; j += 4) *reinterpret_cast<int4*>(dst + j) = make_int4(n[j], n[j + 1], n[j + 2], n[j + 3]);
    }
  }
  {
    const bool multi = live && a.chunk_multi[chunk];
    if (__ballot(multi)) flush_multi_rows<1, KP>(a.ndk_dst, KS, doc, multi, 0, d);
  }
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    int v = d[j];
#pragma unroll
    for (int m = 1; m < oni::kWave; m <<= 1) v += __shfl_xor(v, m);
    d[j] = v;
  }
  if (c == 0) {
#pragma unroll
    for (int j = 0; j < KP; ++j) red[wave][j] = d[j];
  }
  __syncthreads();
  if (threadIdx.x < KS) {
    int v = 0;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) v += red[w][threadIdx.x];
    if (v) atomicAdd(&a.dnk[(int)(blockIdx.x & (unsigned)(a.nk_rep - 1)) * KS + threadIdx.x], v);
  }
}

// ---- ping-pong register sampler (the default sweep kernel) ------------------------------------
// Same numerics as k_gibbs (mul + add weight chain, bitwise identical), restructured for issue
// rate: the loop is unrolled by two so the q row of the next token always lands in the other half
// of a register ping-pong (no per-token 20-wide row copy on a word change, which k_gibbs pays as
// v_cndmask because the change is lane-divergent), and token words/topics (plus MODE-3 word-sorted
// slots) stream two steps ahead so their HBM latency hides behind two steps of math.
template <int G, int KP, int MODE, int P>
__device__ __forceinline__ void pp_step(const OniGibbs& a, int s, int len, int64_t off, int c, int g, int lane,
                                        uint32_t key, uint32_t pos0, uint32_t sweep, int32_t (&n)[KP], oni::U4& r,
                                        uint32_t (&wq)[2], int (&zq)[2], int32_t (&pq)[2], const float (&qc)[KP],
                                        float (&qn)[KP], int& nchg) {
  constexpr int S = oni::kWave / G;
  constexpr int KS = G * KP;
  const int kbase = g * KP;
  const int64_t idx = off + (int64_t)s * S + c;
  const uint32_t w = wq[P];
  const int zo = zq[P];
  const int32_t wp = pq[P];
  if (s + 2 < len) {
    wq[P] = a.tok_word[idx + 2 * S];
    zq[P] = a.tok_z[idx + 2 * S];
    if constexpr (MODE == 3 || MODE == 4) pq[P] = a.wpos[idx + 2 * S];
  }
  if (s + 1 < len && wq[1 - P] != oni::kPadWord) load_row_f<KP>(a.q + (int64_t)wq[1 - P] * KS + kbase, qn);
  if (w == oni::kPadWord) return;  // uniform across the G lanes of a unit
  const uint32_t pos = pos0 + (uint32_t)s;
  if (s == 0 || (pos & 3u) == 0u) r = oni::philox10(oni::U4{pos >> 2, key, sweep, 1u}, a.seed0, a.seed1);
  const uint32_t rr = oni::pick4(r, pos & 3u);
#pragma unroll
  for (int j = 0; j < KP; ++j) n[j] -= (kbase + j == zo);
  float loc[KP];
  float run = 0.f;
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    run = run + ((float)n[j] + a.alpha) * qc[j];
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
    a.tok_z[idx] = (uint8_t)zn;
    if constexpr (MODE == 3) a.z_w[wp] = (uint8_t)zn;
    if constexpr (MODE == 4) mark_changed_w(a, wp, zo, zn);
    if constexpr (MODE == 1) {
      atomicAdd(&a.dnwk[(int64_t)w * KS + zo], -1);
      atomicAdd(&a.dnwk[(int64_t)w * KS + zn], 1);
    }
  }
  if constexpr (MODE == 2) {
    // lane 0 (c = 0) owns the slice's longest chunk, so it is active at every step
    const uint64_t m = __ballot(changed);
    if (lane == 0) a.chg_mask[(off + (int64_t)s * S) / S] = m;
  }
}

template <int G, int KP, int MODE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_gibbs_pp(const OniGibbs a) {
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
  if (live) load_row_i<KP>(a.ndk_src + (int64_t)doc * KS + kbase, n);
  const int len = valid ? a.slice_len[slice] : 0;
  const int64_t off = valid ? a.slice_off[slice] : 0;
  const uint32_t key = live ? a.chunk_key[chunk] : 0u;
  const uint32_t pos0 = live ? (uint32_t)a.chunk_pos0[chunk] : 0u;
  const uint32_t sweep = *a.sweep_ctr;
  oni::U4 r{0, 0, 0, 0};
  int nchg = 0;
  float qa[KP], qb[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) qa[j] = qb[j] = 0.f;
  uint32_t wq[2] = {oni::kPadWord, oni::kPadWord};
  int zq[2] = {0, 0};
  int32_t pq[2] = {0, 0};
  for (int t = 0; t < 2; ++t) {
    if (t < len) {
      wq[t] = a.tok_word[off + t * S + c];
      zq[t] = a.tok_z[off + t * S + c];
      if constexpr (MODE == 3 || MODE == 4) pq[t] = a.wpos[off + t * S + c];
    }
  }
  if (wq[0] != oni::kPadWord) load_row_f<KP>(a.q + (int64_t)wq[0] * KS + kbase, qa);
  for (int s = 0; s < len; s += 2) {
    pp_step<G, KP, MODE, 0>(a, s, len, off, c, g, lane, key, pos0, sweep, n, r, wq, zq, pq, qa, qb, nchg);
    if (s + 1 < len)
      pp_step<G, KP, MODE, 1>(a, s + 1, len, off, c, g, lane, key, pos0, sweep, n, r, wq, zq, pq, qb, qa, nchg);
  }
  if (a.chg_count) add_wave_count(a.chg_count, nchg);
  // ---- epilogue (as k_gibbs): doc rows + per-topic totals --------------------------------------
  int32_t d[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) d[j] = 0;
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

// K ≤ 32 sweep with the doc-topic counts staged in LDS (one lane = one unit, G = 1).
//
// Why: k_gibbs<1,KP> is VALU-issue bound (≈280 vector instructions per token at K = 20, 80 of
// them the compare/select updates n[zo]-- / n[zn]++ of a register row with a per-lane index,
// 20 the int→float converts and 20 the q-row copy on a word change). Here
//  * each lane owns an LDS row a[0..KS) = (float)n_dk (exact integers below 2^24, checked by the
//    host), so the count updates are two single-address LDS read-modify-writes;
//  * the weights form a single fma chain P_j = fma(a_j + α, q_j, P_{j-1}) (the "fma" numerics of
//    the spec, oni355/ref/spec.py gibbs_pass(fma=True)), P kept in registers for the count pass;
//  * the q row of the next token is always prefetched into the other half of a register
//    ping-pong (the loop is unrolled by two), so no per-token row copy is needed.
// Row stride is an odd number of 16-B slots → conflict-free ds_read_b128.
template <int KP>
struct LdsRow {
  static constexpr int kSlots = ((KP / 4) % 2 == 0) ? KP / 4 + 1 : KP / 4;
};

// One token step of k_gibbs_lds. Token words/topics (and MODE-3 word-sorted slots) are
// streamed two steps ahead in a parity-indexed register pair (P is the compile-time parity of s),
// the q row one step ahead into the other half of the q ping-pong.
template <int KP>
__device__ __forceinline__ int count_le(const float (&P)[KP], float excl, float thr);

template <int KP, int MODE, int P, bool AIR>
__device__ __forceinline__ void lds_step(const OniGibbs& a, int s, int len, int64_t off, int lane,
                                         float4* __restrict__ row, PhiloxPair& rng, PendZ& pend,
                                         uint32_t (&wq)[2], int (&zq)[2], int32_t (&pq)[2], const float (&qc)[KP],
                                         float (&qn)[KP], uint64_t* chg_word, int& nchg) {
  constexpr int KS = KP;
  float* rowf = reinterpret_cast<float*>(row);
  const int64_t idx = off + (int64_t)s * 64 + lane;
  const uint32_t w = wq[P];
  const int zo = zq[P];
  const int32_t wp = pq[P];
  if (s + 2 < len) {
    wq[P] = a.tok_word[idx + 128];
    zq[P] = a.tok_z[idx + 128];
    if constexpr (MODE == 3 || MODE == 4) pq[P] = a.wpos[idx + 128];
  }
  if (s + 1 < len && wq[1 - P] != oni::kPadWord) load_row_f<KP>(a.q + (int64_t)wq[1 - P] * KS, qn);
  flush_pend<MODE>(a, pend, KS);  // the previous step's stores, behind this step's loads
  rng.step(s, a);
  bool changed = false;
  if (w != oni::kPadWord) {
    const uint32_t rr = rng.pick(s);
    rowf[zo] = rowf[zo] - 1.0f;
    float Pc[KP];
    float run = 0.f;
#pragma unroll
    for (int j = 0; j < KP / 4; ++j) {
      const float4 av = row[j];
      run = fmaf(AIR ? av.x : av.x + a.alpha, qc[4 * j + 0], run);
      Pc[4 * j + 0] = run;
      run = fmaf(AIR ? av.y : av.y + a.alpha, qc[4 * j + 1], run);
      Pc[4 * j + 1] = run;
      run = fmaf(AIR ? av.z : av.z + a.alpha, qc[4 * j + 2], run);
      Pc[4 * j + 2] = run;
      run = fmaf(AIR ? av.w : av.w + a.alpha, qc[4 * j + 3], run);
      Pc[4 * j + 3] = run;
    }
    const float thr = oni::u01(rr) * run;
    const int cnt = count_le<KP>(Pc, 0.f, thr);  // 0 + P_j == P_j: the same compares
    const int zn = cnt < a.K - 1 ? cnt : a.K - 1;
    rowf[zn] = rowf[zn] + 1.0f;
    changed = zn != zo;
    nchg += changed;
    if (changed) {
      pend.on = true;
      pend.idx = idx;
      pend.zo = zo;
      pend.zn = zn;
      pend.pw = wp;
      pend.w = w;
    }
  }
  if constexpr (MODE == 2) {
    const uint64_t m = __ballot(changed);
    if (lane == 0) {
      pend.m = m;
      pend.mdst = chg_word + s;
    }
  }
}

template <int KP, int MODE, bool AIR = false>
__global__ __launch_bounds__(kBlock) void k_gibbs_lds(const OniGibbs a) {
  constexpr int KS = KP;
  constexpr int kSlots = LdsRow<KP>::kSlots;
  __shared__ float4 sa[kBlock * kSlots];
  __shared__ int32_t red[kWavesPerBlock][KS];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t slice = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const bool valid = slice < a.n_slices;
  const int64_t chunk = slice * 64 + lane;
  const int doc = valid ? a.chunk_doc[chunk] : -1;
  const bool live = doc >= 0;
  float4* row = sa + threadIdx.x * kSlots;
  {
    int32_t n0[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) n0[j] = 0;
    if (live) load_row_i<KP>(a.ndk_src + (int64_t)doc * KS, n0);
    const float a0 = AIR ? a.alpha : 0.f;  // AIR: rows hold n + α (see k_gibbs_ldsg)
#pragma unroll
    for (int j = 0; j < KP / 4; ++j)
      row[j] = make_float4((float)n0[4 * j] + a0, (float)n0[4 * j + 1] + a0, (float)n0[4 * j + 2] + a0,
                           (float)n0[4 * j + 3] + a0);
  }
  const int len = valid ? a.slice_len[slice] : 0;
  const int64_t off = valid ? a.slice_off[slice] : 0;
  const uint32_t key = live ? a.chunk_key[chunk] : 0u;
  const uint32_t pos0 = live ? (uint32_t)a.chunk_pos0[chunk] : 0u;
  const uint32_t sweep = *a.sweep_ctr;
  uint64_t* chg_word = MODE == 2 ? a.chg_mask + off / 64 : nullptr;
  PhiloxPair rng;
  rng.init(pos0, key, sweep, 1u, a);
  PendZ pend;
  float qa[KP], qb[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) qa[j] = qb[j] = 0.f;
  int nchg = 0;
  uint32_t wq[2] = {oni::kPadWord, oni::kPadWord};
  int zq[2] = {0, 0};
  int32_t pq[2] = {0, 0};
  for (int t = 0; t < 2; ++t) {
    if (t < len) {
      wq[t] = a.tok_word[off + t * 64 + lane];
      zq[t] = a.tok_z[off + t * 64 + lane];
      if constexpr (MODE == 3 || MODE == 4) pq[t] = a.wpos[off + t * 64 + lane];
    }
  }
  if (wq[0] != oni::kPadWord) load_row_f<KP>(a.q + (int64_t)wq[0] * KS, qa);
  for (int s = 0; s < len; s += 2) {
    lds_step<KP, MODE, 0, AIR>(a, s, len, off, lane, row, rng, pend, wq, zq, pq, qa, qb, chg_word, nchg);
    if (s + 1 < len)
      lds_step<KP, MODE, 1, AIR>(a, s + 1, len, off, lane, row, rng, pend, wq, zq, pq, qb, qa, chg_word, nchg);
  }
  flush_pend<MODE>(a, pend, KS);
  if (a.chg_count) add_wave_count(a.chg_count, nchg);
  // epilogue: counts back to ints, doc rows, per-topic totals (n0 re-read: keeps it out of VGPRs)
  const float* rowf = reinterpret_cast<const float*>(row);
  int32_t d[KP], n[KP], n0[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) n0[j] = 0;
  if (live) load_row_i<KP>(a.ndk_src + (int64_t)doc * KS, n0);
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    n[j] = (int32_t)(AIR ? rowf[j] - a.alpha : rowf[j]);
    d[j] = n[j] - n0[j];
  }
  const bool multi = live && a.chunk_multi[chunk];
  if (live && !multi) {
    int32_t* dst = a.ndk_dst + (int64_t)doc * KS;
#pragma unroll
    for (int j = 0; j < KP; j += 4) *reinterpret_cast<int4*>(dst + j) = make_int4(n[j], n[j + 1], n[j + 2], n[j + 3]);
  }
  if (__ballot(multi)) flush_multi_rows<1, KP>(a.ndk_dst, KS, doc, multi, 0, d);
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    int v = d[j];
#pragma unroll
    for (int m = 1; m < oni::kWave; m <<= 1) v += __shfl_xor(v, m);
    d[j] = v;
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < KP; ++j) red[wave][j] = d[j];
  }
  __syncthreads();
  if (threadIdx.x < KS) {
    int v = 0;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) v += red[w][threadIdx.x];
    if (v) atomicAdd(&a.dnk[(int)(blockIdx.x & (unsigned)(a.nk_rep - 1)) * KS + threadIdx.x], v);
  }
}

// ---- multi-lane units (K > 32) with LDS-staged counts ------------------------------------------
// k_gibbs<G>1> is VALU-issue bound (measured at K = 100: ≈1250 SIMD cycles per wave step, i.e.
// ≈250 vector instructions for the 8 tokens a wave samples per step). Per lane and per topic slot
// it spends ≈11 instructions: a compare/select pair for each of n[zo]-- and n[zn]++ (register
// rows can only be indexed by select chains), convert + add + mul + add for the weight, and
// add + compare + select to count the prefix entries below the threshold. Here
//  * lane (unit c, g) keeps its KP counts as f32 in a private LDS row, so each count update is one
//    ds_add_f32 by the owning lane (exact integers below 2^24, checked by the host);
//  * the weights form an fma chain P_j = fma(n_j + α, q_j, P_{j-1}) inside the lane (the spec's
//    "fma" numerics, oni355/ref/spec.py gibbs_pass(fma=True), extended to G > 1) followed by the
//    same cross-lane Hillis-Steele scan as k_gibbs;
//  * the count #{j : excl + P_j ≤ thr} is a branch-free binary search over the lane's monotone
//    prefix (5 compares + 11 selects for KP = 16 instead of 16 compare/add pairs) — exact because
//    fl(excl + x) is monotone in x.
// ≈2× fewer VALU instructions per token; bitwise equal to the fma oracle.
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

// Sum of an int over each aligned group of G ∈ {2, 4, 8, 16} lanes with DPP butterflies (no LDS
// crossbar round trip): quad_perm swaps for 1 and 2, half-row / row mirrors for 4 and 8 (after the
// lower levels every lane of a sub-group holds the sub-group sum, so any cross pairing works).
template <int G>
__device__ __forceinline__ int group_sum_dpp(int v) {
  static_assert(G == 2 || G == 4 || G == 8 || G == 16, "DPP group sums need G in {2, 4, 8, 16}");
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
  if constexpr (G >= 4) v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
  if constexpr (G >= 8) v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, true);  // row_half_mirror
  if constexpr (G >= 16) v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, true);  // row_mirror
  return v;
}

// Float Hillis-Steele inclusive scan over aligned groups of G ≤ 16 lanes with DPP row shifts:
// the same additions in the same order as the __shfl_up scan (bitwise identical), without LDS
// crossbar round trips. Groups never straddle a 16-lane DPP row.
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

// QP = 1: the q row of the next token is prefetched one step ahead (token words stream two steps
// ahead so the prefetch address is known early) and copied in on a word change; QP = 0 loads the
// row when the word changes.
// AIR: the LDS rows hold n_dk + α instead of n_dk (the host sets it only when every n + α of this
// corpus is exact in f32, e.g. α = 50/K ∈ {2.5, 1, 0.5} with documents below 2^22 tokens), which
// drops the per-topic "+ α" from the inner product -- same values, bitwise the same draws.
// OCC: minimum waves per SIMD the register allocation must allow (1 = the compiler's default,
// which lands at 98 VGPRs / 4 waves for (4, 28); 5 = 96 VGPRs, the LDS limit of 30.4 KB blocks).
template <int G, int KP, int MODE, int QP, bool AIR = false, int OCC = 1>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void k_gibbs_ldsg(const OniGibbs a) {
  static_assert(G > 1, "G = 1 uses k_gibbs_lds");
  constexpr int S = oni::kWave / G;
  constexpr int KS = G * KP;
  constexpr int kSlots = LdsRow<KP>::kSlots;
  __shared__ float4 sa[kBlock * kSlots];
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
  float4* row = sa + threadIdx.x * kSlots;
  float* rowf = reinterpret_cast<float*>(row);
  {
    int32_t n0[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) n0[j] = 0;
    if (live) load_row_i<KP>(a.ndk_src + (int64_t)doc * KS + kbase, n0);
    const float a0 = AIR ? a.alpha : 0.f;
#pragma unroll
    for (int j = 0; j < KP / 4; ++j)
      row[j] = make_float4((float)n0[4 * j] + a0, (float)n0[4 * j + 1] + a0, (float)n0[4 * j + 2] + a0,
                           (float)n0[4 * j + 3] + a0);
  }
  const int len = valid ? a.slice_len[slice] : 0;
  const int64_t off = valid ? a.slice_off[slice] : 0;
  const uint32_t key = live ? a.chunk_key[chunk] : 0u;
  const uint32_t pos0 = live ? (uint32_t)a.chunk_pos0[chunk] : 0u;
  const uint32_t sweep = *a.sweep_ctr;
  // Philox blocks are shared by the unit: lane g holds the block of 4-token group gbase + g, so
  // the unit computes one block per G·4 tokens instead of every lane computing one per 4 tokens
  // (the 36 quarter-rate integer multiplies of a block were ≈30 % of the sampler's issue slots)
  //
  // The refresh is wave-uniform: every kRefresh = 4G - 3 steps each unit recomputes the G blocks
  // that cover its next kRefresh tokens (any alignment of pos0 fits in G groups). A per-unit
  // refresh (when the token leaves the unit's G groups) is taken by SOME unit of the wave on most
  // steps -- 64 % of them at G = 4, 99 % at G = 2 -- and a block costs 36 quarter-rate multiplies
  // whoever is masked off; the same blocks at a uniform cadence give the same draws bitwise.
  constexpr int kRefresh = 4 * G - 3;
  uint32_t gbase = pos0 >> 2;
  oni::U4 r = oni::philox10(oni::U4{gbase + (uint32_t)g, key, sweep, 1u}, a.seed0, a.seed1);
  int next_refresh = kRefresh;
  uint32_t wprev = oni::kPadWord;
  float qv[KP], qn[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) qv[j] = qn[j] = 0.f;
  int nchg = 0;
  uint32_t w_nx = len > 0 ? a.tok_word[off + c] : oni::kPadWord;
  int z_nx = len > 0 ? (int)a.tok_z[off + c] : 0;
  uint32_t w_nx2 = (QP && len > 1) ? a.tok_word[off + S + c] : oni::kPadWord;
  if (QP && w_nx != oni::kPadWord) load_row_f<KP>(a.q + (int64_t)w_nx * KS + kbase, qn);
  // Deferred bookkeeping: a changed token's stores/atomics are issued in the NEXT step, right
  // after that step's token-stream loads. Every vector-memory op retires through the wave's in-order vmcnt
  // counter, so a store issued at the end of a step made the step's closing wait (for the next
  // token's word/topic) wait out a full store round trip as well; issued a step later, it drains
  // behind the step's math. MODE 3/4 stream the word-sorted slot with the token (WPF) instead
  // of loading it after the draw. Nothing in the kernel reads these locations: same results.
  constexpr bool WPF = MODE == 3 || MODE == 4;
  int32_t p_nx = (WPF && len > 0) ? a.wpos[off + c] : 0;
  bool pend = false;
  int64_t p_idx = 0;
  int p_zo = 0, p_zn = 0;
  int32_t p_pw = 0;
  uint32_t p_w = 0;
  uint64_t p_m = 0;
  int64_t p_mi = -1;
  auto flush = [&]() {
    if (pend) {
      a.tok_z[p_idx] = (uint8_t)p_zn;
      if constexpr (MODE == 3) a.z_w[p_pw] = (uint8_t)p_zn;
      if constexpr (MODE == 4) mark_changed_w(a, p_pw, p_zo, p_zn);
      if constexpr (MODE == 1) {
        atomicAdd(&a.dnwk[(int64_t)p_w * KS + p_zo], -1);
        atomicAdd(&a.dnwk[(int64_t)p_w * KS + p_zn], 1);
      }
      pend = false;
    }
    if constexpr (MODE == 2) {
      if (p_mi >= 0) a.chg_mask[p_mi] = p_m;
      p_mi = -1;
    }
  };
  for (int s = 0; s < len; ++s) {
    const int64_t idx = off + (int64_t)s * S + c;
    const uint32_t w = w_nx;
    const int zo = z_nx;
    const int32_t pw = p_nx;
    if (WPF && s + 1 < len) p_nx = a.wpos[idx + S];
    if constexpr (QP) {
      w_nx = w_nx2;
      if (s + 1 < len) z_nx = a.tok_z[idx + S];
      if (s + 2 < len) w_nx2 = a.tok_word[idx + 2 * S];
      if (w != wprev) {
#pragma unroll
        for (int j = 0; j < KP; ++j) qv[j] = qn[j];
        wprev = w;
      }
      if (s + 1 < len && w_nx != w && w_nx != oni::kPadWord) load_row_f<KP>(a.q + (int64_t)w_nx * KS + kbase, qn);
    } else if (s + 1 < len) {
      w_nx = a.tok_word[idx + S];
      z_nx = a.tok_z[idx + S];
    }
    flush();  // after the token-stream loads: their wait at the step's end covers a store that had the whole step
    if (s == next_refresh) {  // wave-uniform (before the pad test: every lane takes it together)
      next_refresh += kRefresh;
      gbase = (pos0 + (uint32_t)s) >> 2;
      r = oni::philox10(oni::U4{gbase + (uint32_t)g, key, sweep, 1u}, a.seed0, a.seed1);
    }
    if (w == oni::kPadWord) continue;  // uniform across the G lanes of a unit
    const uint32_t pos = pos0 + (uint32_t)s;
    const uint32_t gi = pos >> 2;
    const uint32_t rr = (uint32_t)__shfl((int)oni::pick4(r, pos & 3u), (int)(gi - gbase), G);
    const unsigned zlo = (unsigned)(zo - kbase);
    if (zlo < (unsigned)KP) rowf[zlo] -= 1.0f;
    if (!QP && w != wprev) {
      load_row_f<KP>(a.q + (int64_t)w * KS + kbase, qv);
      wprev = w;
    }
    float P[KP];
    float run = 0.f;
#pragma unroll
    for (int j = 0; j < KP / 4; ++j) {
      const float4 av = row[j];
      run = fmaf(AIR ? av.x : av.x + a.alpha, qv[4 * j + 0], run);
      P[4 * j + 0] = run;
      run = fmaf(AIR ? av.y : av.y + a.alpha, qv[4 * j + 1], run);
      P[4 * j + 1] = run;
      run = fmaf(AIR ? av.z : av.z + a.alpha, qv[4 * j + 2], run);
      P[4 * j + 2] = run;
      run = fmaf(AIR ? av.w : av.w + a.alpha, qv[4 * j + 3], run);
      P[4 * j + 3] = run;
    }
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
      pend = true;
      p_idx = idx;
      p_zo = zo;
      p_zn = zn;
      p_pw = pw;
      p_w = w;
    }
    if constexpr (MODE == 2) {
      // lane 0 (c = 0) owns the slice's longest chunk, so it is active at every step
      const uint64_t m = __ballot(changed);
      if (lane == 0) {
        p_m = m;
        p_mi = (off + (int64_t)s * S) / S;
      }
    }
  }
  flush();
  if (a.chg_count) add_wave_count(a.chg_count, nchg);
  // ---- epilogue (as k_gibbs): doc rows + per-topic totals ----------------------------------------
  int32_t d[KP], n[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    n[j] = (int32_t)(AIR ? rowf[j] - a.alpha : rowf[j]);
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

template <int G, int KP>
int launch_gibbs(const OniGibbs& a, bool init, int mode, int qpf, hipStream_t s) {
  // qpf (sampler variant): 1 = k_gibbs_pp (ping-pong register sampler, default), 0 = k_gibbs with
  // a q-row load on each word change, 4 = k_gibbs with one-step q prefetch + row copy,
  // 2 = k_gibbs_lds (G = 1) / k_gibbs_ldsg (G > 1): LDS-staged counts, fma numerics
  if (a.KS != G * KP || mode < 0 || mode > 4) return (int)hipErrorInvalidValue;
  if (G == 1 && qpf == 5) qpf = 2;  // q-prefetching LDS sampler is the multi-lane variant
  if (G > 1 && qpf == 6) qpf = 4;   // the two-deep stream variant is written for G = 1
  // qpf 7 = DZ (LDS-staged topics, deferred bookkeeping): G = 1 sweeps of slices ≤ kDzMaxLen steps
  // in MODE 0/1/3/4; the caller guarantees the slice bound (slice_len[0] is the longest)
  if (qpf == 7 && (G != 1 || init || mode == 2)) qpf = 4;
  if (qpf == 8 && (G != 1 || init || mode == 2)) qpf = G == 1 ? 6 : 4;  // 8 = k_gibbs_q2 + DZ
  // qpf 9 = k_gibbs_ldsg with a 5-wave register budget (G > 1, recount / wdelta sweeps)
  if (qpf == 9 && (G == 1 || init || (mode != 0 && mode != 4))) qpf = 2;
  const unsigned grid = (unsigned)((a.n_slices + kWavesPerBlock - 1) / kWavesPerBlock);
  if (grid == 0) return 0;
  if constexpr (G == 1) {
    if (qpf == 8) {
      switch (mode) {
        case 0: k_gibbs_q2<KP, 0, true><<<grid, kBlock, 0, s>>>(a); break;
        case 1: k_gibbs_q2<KP, 1, true><<<grid, kBlock, 0, s>>>(a); break;
        case 3: k_gibbs_q2<KP, 3, true><<<grid, kBlock, 0, s>>>(a); break;
        default: k_gibbs_q2<KP, 4, true><<<grid, kBlock, 0, s>>>(a); break;
      }
      return (int)hipGetLastError();
    }
    if (qpf == 7) {
      switch (mode) {
        case 0: k_gibbs<1, KP, false, 0, true, true><<<grid, kBlock, 0, s>>>(a); break;
        case 1: k_gibbs<1, KP, false, 1, true, true><<<grid, kBlock, 0, s>>>(a); break;
        case 3: k_gibbs<1, KP, false, 3, true, true><<<grid, kBlock, 0, s>>>(a); break;
        default: k_gibbs<1, KP, false, 4, true, true><<<grid, kBlock, 0, s>>>(a); break;
      }
      return (int)hipGetLastError();
    }
    if (!init && qpf == 6) {
      switch (mode) {
        case 0: k_gibbs_q2<KP, 0><<<grid, kBlock, 0, s>>>(a); break;
        case 1: k_gibbs_q2<KP, 1><<<grid, kBlock, 0, s>>>(a); break;
        case 2: k_gibbs_q2<KP, 2><<<grid, kBlock, 0, s>>>(a); break;
        case 3: k_gibbs_q2<KP, 3><<<grid, kBlock, 0, s>>>(a); break;
        default: k_gibbs_q2<KP, 4><<<grid, kBlock, 0, s>>>(a); break;
      }
      return (int)hipGetLastError();
    }
  }
  if (init) {
    // mode 1: n_wk by per-token atomics (same-address contention on frequent words: 1.5 ms at 25M
    // tokens); mode 0: no n_wk bookkeeping, the caller rebuilds it with the word-sorted recount
    if (mode == 0) k_gibbs<G, KP, true, 0, false><<<grid, kBlock, 0, s>>>(a);
    else k_gibbs<G, KP, true, 1, false><<<grid, kBlock, 0, s>>>(a);
    return (int)hipGetLastError();
  }
  if constexpr (G > 1) {
    if (qpf == 9) {
      if (mode == 4) {
        if (a.flags & 1) k_gibbs_ldsg<G, KP, 4, 0, true, 5><<<grid, kBlock, 0, s>>>(a);
        else k_gibbs_ldsg<G, KP, 4, 0, false, 5><<<grid, kBlock, 0, s>>>(a);
      } else if (a.flags & 1) {
        k_gibbs_ldsg<G, KP, 0, 0, true, 5><<<grid, kBlock, 0, s>>>(a);
      } else {
        k_gibbs_ldsg<G, KP, 0, 0, false, 5><<<grid, kBlock, 0, s>>>(a);
      }
      return (int)hipGetLastError();
    }
  }
  if (mode == 4) {  // word-sorted change bitmap
    if constexpr (G > 1) {
      if (qpf == 2 || qpf == 5) {
        if (qpf == 5) k_gibbs_ldsg<G, KP, 4, 1><<<grid, kBlock, 0, s>>>(a);
        else if (a.flags & 1) k_gibbs_ldsg<G, KP, 4, 0, true><<<grid, kBlock, 0, s>>>(a);
        else k_gibbs_ldsg<G, KP, 4, 0><<<grid, kBlock, 0, s>>>(a);
        return (int)hipGetLastError();
      }
    } else {
      if (qpf == 2) {
        if (a.flags & 1) k_gibbs_lds<KP, 4, true><<<grid, kBlock, 0, s>>>(a);
        else k_gibbs_lds<KP, 4><<<grid, kBlock, 0, s>>>(a);
        return (int)hipGetLastError();
      }
    }
    if (qpf == 4) k_gibbs<G, KP, false, 4, true><<<grid, kBlock, 0, s>>>(a);
    else if (qpf == 1) k_gibbs_pp<G, KP, 4><<<grid, kBlock, 0, s>>>(a);
    else if (qpf == 0) k_gibbs<G, KP, false, 4, false><<<grid, kBlock, 0, s>>>(a);
    else return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
  }
  if constexpr (G == 1) {
    if (qpf == 2) {
      if (a.flags & 1) {
        if (mode == 0) k_gibbs_lds<KP, 0, true><<<grid, kBlock, 0, s>>>(a);
        else if (mode == 1) k_gibbs_lds<KP, 1, true><<<grid, kBlock, 0, s>>>(a);
        else if (mode == 2) k_gibbs_lds<KP, 2, true><<<grid, kBlock, 0, s>>>(a);
        else k_gibbs_lds<KP, 3, true><<<grid, kBlock, 0, s>>>(a);
      } else if (mode == 0) k_gibbs_lds<KP, 0><<<grid, kBlock, 0, s>>>(a);
      else if (mode == 1) k_gibbs_lds<KP, 1><<<grid, kBlock, 0, s>>>(a);
      else if (mode == 2) k_gibbs_lds<KP, 2><<<grid, kBlock, 0, s>>>(a);
      else k_gibbs_lds<KP, 3><<<grid, kBlock, 0, s>>>(a);
      return (int)hipGetLastError();
    }
  } else {
    if (qpf == 2) {
      if (a.flags & 1) {
        if (mode == 0) k_gibbs_ldsg<G, KP, 0, 0, true><<<grid, kBlock, 0, s>>>(a);
        else if (mode == 1) k_gibbs_ldsg<G, KP, 1, 0, true><<<grid, kBlock, 0, s>>>(a);
        else if (mode == 2) k_gibbs_ldsg<G, KP, 2, 0, true><<<grid, kBlock, 0, s>>>(a);
        else k_gibbs_ldsg<G, KP, 3, 0, true><<<grid, kBlock, 0, s>>>(a);
      } else if (mode == 0) k_gibbs_ldsg<G, KP, 0, 0><<<grid, kBlock, 0, s>>>(a);
      else if (mode == 1) k_gibbs_ldsg<G, KP, 1, 0><<<grid, kBlock, 0, s>>>(a);
      else if (mode == 2) k_gibbs_ldsg<G, KP, 2, 0><<<grid, kBlock, 0, s>>>(a);
      else k_gibbs_ldsg<G, KP, 3, 0><<<grid, kBlock, 0, s>>>(a);
      return (int)hipGetLastError();
    }
    if (qpf == 5) {
      if (mode == 0) k_gibbs_ldsg<G, KP, 0, 1><<<grid, kBlock, 0, s>>>(a);
      else if (mode == 1) k_gibbs_ldsg<G, KP, 1, 1><<<grid, kBlock, 0, s>>>(a);
      else if (mode == 2) k_gibbs_ldsg<G, KP, 2, 1><<<grid, kBlock, 0, s>>>(a);
      else k_gibbs_ldsg<G, KP, 3, 1><<<grid, kBlock, 0, s>>>(a);
      return (int)hipGetLastError();
    }
  }
  if (qpf == 4) {  // one-step q-row prefetch (any unit width)
    if (mode == 0) k_gibbs<G, KP, false, 0, true><<<grid, kBlock, 0, s>>>(a);
    else if (mode == 1) k_gibbs<G, KP, false, 1, true><<<grid, kBlock, 0, s>>>(a);
    else if (mode == 2) k_gibbs<G, KP, false, 2, true><<<grid, kBlock, 0, s>>>(a);
    else k_gibbs<G, KP, false, 3, true><<<grid, kBlock, 0, s>>>(a);
    return (int)hipGetLastError();
  }
  if (qpf == 1) {
    if (mode == 0) k_gibbs_pp<G, KP, 0><<<grid, kBlock, 0, s>>>(a);
    else if (mode == 1) k_gibbs_pp<G, KP, 1><<<grid, kBlock, 0, s>>>(a);
    else if (mode == 2) k_gibbs_pp<G, KP, 2><<<grid, kBlock, 0, s>>>(a);
    else k_gibbs_pp<G, KP, 3><<<grid, kBlock, 0, s>>>(a);
    return (int)hipGetLastError();
  }
  if (mode == 0) k_gibbs<G, KP, false, 0, false><<<grid, kBlock, 0, s>>>(a);
  else if (mode == 1) k_gibbs<G, KP, false, 1, false><<<grid, kBlock, 0, s>>>(a);
  else if (mode == 2) k_gibbs<G, KP, false, 2, false><<<grid, kBlock, 0, s>>>(a);
  else k_gibbs<G, KP, false, 3, false><<<grid, kBlock, 0, s>>>(a);
  return (int)hipGetLastError();
}

}  // namespace

// Per-unit-width dispatchers (gibbs_g1.hip, gibbs_g2.hip, gibbs_g4.hip, gibbs_g8.hip): launch
// launch_gibbs<G, KP> for a supported KP; hipErrorInvalidValue otherwise.
int oni_gibbs_dispatch_g1(const OniGibbs& a, int KP, bool init, int mode, int qpf, hipStream_t s);
int oni_gibbs_dispatch_g2(const OniGibbs& a, int KP, bool init, int mode, int qpf, hipStream_t s);
int oni_gibbs_dispatch_g4(const OniGibbs& a, int KP, bool init, int mode, int qpf, hipStream_t s);
int oni_gibbs_dispatch_g8(const OniGibbs& a, int G, int KP, bool init, int mode, int qpf, hipStream_t s);
