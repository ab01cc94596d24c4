// K10-MH -- Metropolis-Hastings LDA sweep with sweep-static alias proposals (k_gibbs_mh), its
// proposal-table builder (k_mh_alias) and the one-lane init pass for K > 32 (k_gibbs_mh_init).
//
// Why: the dense samplers spend K multiply-adds (plus a scan and a search) on every token; at
// K = 100 k_gibbs_ldsg runs 0.89 ms per 25M-token sweep, bound by the per-token q-row round trip
// and its 4-lane scans (docs/performance.md). An MH step costs O(1) per token whatever K is: the
// word proposal ∝ q[w, ·] is a two-level inverse CDF -- a 64-B row of bucket prefix sums built once
// per sweep (k_mh_cdf: a streaming pass over q, V·64 B written), then the bucket's own 8-16 q values
// -- and the doc proposal an alias table of the sweep-start row of every document spread over
// several chunks; the acceptance test needs a handful of counts. (Round 4 built a Vose alias table
// of every word's q row per sweep: V·K·16 B of records, 0.24 ms at V = 180k, K = 100, sequential
// per-lane construction bound by LDS latency.) Semantics and numerics: oni355/ref/spec.py
// gibbs_pass_mh / mh_moves / alias_table, replayed bit for bit (tests/test_gpu_mh.py); the moves
// leave the collapsed conditional invariant (tests/test_mh_conditional.py).
//
// Execution model (MI355X-first):
//  * One lane per chunk (S = 64 chunks per SELL slice, one wave per block): the lane walks its
//    chunk sequentially. Its doc counts live in LDS as u8 cells, interleaved by lane
//    (cell k of lane l at byte k*64 + l: any per-lane topic index hits a distinct dword column);
//    a one-chunk document keeps n_dk (≤ 127), a multi-chunk one keeps n − n_src + 128 (chunks are
//    ≤ 127 tokens), so 100 topics cost 6.4 KB per wave instead of 25.6 KB of f32 rows. The
//    chunk's current topics (the one-chunk doc proposal picks a random other token) sit next to
//    them, also u8 and interleaved.
//  * Loads are software-pipelined by token: the token word four steps ahead (CDF proposal; two
//    with the alias records), the level-1 CDF row two steps ahead; the next token's Philox block,
//    q[w, zo], the bucket's q values, its alias entry (and a multi-chunk doc's alias entry and
//    n_src[zo]) one step ahead -- all independent of the chain state -- so a step waits only for
//    the gathers that depend on its proposals (q[w, t], n_src[t]).
//  * The texture-address unit is this kernel's busiest (~75 % at the config-5 flow share,
//    profiles/r6/mh_pmc/): a scattered load costs it about a cycle per distinct line, so the 64-B
//    level-1 rows are gathered four lanes per row (16 lines per load instead of 64) and turned back
//    to one row per lane through LDS (4.30 → 4.16 ms per config-5 sweep with the deeper word
//    pipeline, profiles/r6/mh_coop/; the buckets gathered the same way lost: their LDS round trip
//    sits in the step's dependency chain).
//  * Every draw is Philox4x32-10 on (pos, doc key, sweep, 2 + move): a pure function of the data
//    and the seed, so the chain is bitwise identical for any GPU count or chunk placement.
#include "gibbs_sampler.h"

struct OniMH {
  OniGibbs g;
  const uint4* walias;         // [V][K] alias word proposal records {thr24 << 8 | alias, q_j, q_alias, Σ q} (wp 0)
  const float* wsum;           // [V] Σ_k q[w, k] (wp 0)
  const float* wcdf;           // [V][16] level-1 CDF rows of the word proposal ∝ q[w, ·] (wp 8 / 16, k_mh_cdf)
  const uint32_t* dalias;      // [n_long][K] alias entries of the multi-chunk docs' n_src + α
  const float* mh_g;           // [KS] 1 / (n_k + Vβ + 1)
  const int32_t* chunk_dslot;  // [C] row of dalias (multi-chunk doc) or -1
  const int32_t* chunk_len;    // [C] tokens of the chunk
  float kalpha;                // f32(K) · α
  float inv_alpha;             // f32(1/α)
  int32_t lmax;                // longest chunk (LDS topic slice rows)
  int32_t doc_moves;           // 1 or 2
  int32_t wp;                  // word proposal: 0 alias records, 8 / 16 two-level CDF (bucket width)
};

namespace {

constexpr int kMHBias = 128;
constexpr int kAS = 65;  // k_mh_alias LDS row stride (dwords)

// j = ⌊r·K / 2^32⌋ and the coin (top 24 bits of the low word) of an alias draw
__device__ __forceinline__ void alias_index(uint32_t r, int K, int& j, uint32_t& coin) {
  const uint64_t p = (uint64_t)r * (uint32_t)K;
  j = (int)(p >> 32);
  coin = (uint32_t)p >> 8;
}
__device__ __forceinline__ int alias_resolve(int j, uint32_t coin, uint32_t e) {
  return coin < (e >> 8) ? j : (int)(e & 0xFFu);
}

// ---- proposal tables ---------------------------------------------------------------------------
// One lane per row (rows [0, V): word rows of q; rows [V, V + n_long): sweep-start rows of the
// multi-chunk docs + α). Sequential f32 per lane, exactly spec.alias_table: sum, scale, classify
// into the small / large stacks (one u8 array: small grows up from 0, large down from K − 1),
// pair off, leftovers keep their own index. The rows are read and written cooperatively (the wave
// walks its 64 rows, lanes along k: coalesced), p / entries / stack live in LDS transposed to
// [k][row] for the per-lane sequential part.
// Word rows (the alias word proposal, small vocabularies) are written as 16-B records {entry, q_j,
// q_alias(j), Σ_k q_k}: the sampler's one gather of a word proposal then also brings q_t and the row
// sum (the word move's ratio), so a token costs three scattered loads (record, q[w, zo], q[w, t_doc])
// instead of five. With V = 0 only the documents' rows (and g) are built (the CDF word proposal).
__global__ __launch_bounds__(64) void k_mh_alias(const float* __restrict__ q, int64_t V, int K, int KS,
                                                  const int32_t* __restrict__ ndk, const int32_t* __restrict__ rows,
                                                  int64_t n_long, float alpha, uint4* __restrict__ wrec,
                                                  float* __restrict__ wsum, uint32_t* __restrict__ dalias,
                                                  const int32_t* __restrict__ nk, float vbeta, float* __restrict__ g,
                                                  bool coal) {
  extern __shared__ __align__(16) unsigned char smem_alias[];
  // p is [K][65], one column per lane. The entries share its storage: Vose writes entry s once
  // p[s] is spent (s is the popped small, whose weight is already in a register, or the carried
  // large, whose weight lives in a register), and the leftovers get their own index after the
  // pairing; 32 instead of 58 KB per wave at K = 100 (4 waves per CU instead of 2)
  float* p = reinterpret_cast<float*>(smem_alias);
  uint32_t* ent = reinterpret_cast<uint32_t*>(smem_alias);
  float* tots = reinterpret_cast<float*>(smem_alias + (size_t)K * kAS * sizeof(float));   // [64]
  uint8_t* stk = smem_alias + (size_t)K * kAS * sizeof(float) + 64 * sizeof(float);      // [K][64]
  const int lane = threadIdx.x;
  if (blockIdx.x == 0) {
    for (int k = lane; k < KS; k += 64) g[k] = 1.0f / (((float)nk[k] + vbeta) + 1.0f);
  }
  const int64_t r0 = (int64_t)blockIdx.x * 64;
  const int nrows = (int)((V + n_long - r0) < 64 ? (V + n_long - r0) : 64);
  // each lane loads its own row (16-B vectors; K rows of q are KS-strided, KS % 4 == 0)
  const int64_t row = r0 + lane;
  const bool has = lane < nrows;
  const bool word = has && row < V;
  const float* qr = q + (word ? row : 0) * KS;
  const int32_t* br = ndk + (has && !word ? (int64_t)rows[row - V] : 0) * KS;
  if (has) {
#pragma unroll 4
    for (int k = 0; k < K; k += 4) {
      float4 v;
      if (word) {
        v = *reinterpret_cast<const float4*>(qr + k);
      } else {
        const int4 c = *reinterpret_cast<const int4*>(br + k);
        v = make_float4((float)c.x + alpha, (float)c.y + alpha, (float)c.z + alpha, (float)c.w + alpha);
      }
      p[k * kAS + lane] = v.x;
      if (k + 1 < K) p[(k + 1) * kAS + lane] = v.y;
      if (k + 2 < K) p[(k + 2) * kAS + lane] = v.z;
      if (k + 3 < K) p[(k + 3) * kAS + lane] = v.w;
    }
  }
  __syncthreads();
  if (lane < nrows) {
    float tot = 0.f;
    for (int k = 0; k < K; ++k) tot = tot + p[k * kAS + lane];
    tots[lane] = tot;
    const float scale = (float)K / tot;
    int ns = 0, nl = 0;
    for (int k = 0; k < K; ++k) {
      const float v = p[k * kAS + lane] * scale;
      p[k * kAS + lane] = v;
      if (v < 1.0f) stk[(ns++) * 64 + lane] = (uint8_t)k;
      else stk[(K - 1 - nl++) * 64 + lane] = (uint8_t)k;
    }
    // Vose pairing. The large index l of a pair is pushed back and popped again by the very next
    // pair (onto the small stack if its weight fell below 1, else onto the large one), so it is
    // carried in registers with its weight: one stack read and one weight read per pair.
    if (ns > 0 && nl > 0) {
      int s = stk[(--ns) * 64 + lane];
      float ps = p[s * kAS + lane];
      int l = stk[(K - nl) * 64 + lane];
      --nl;
      float pl = p[l * kAS + lane];
      // branch-free: lanes pair at their own pace without splitting the wave's paths
      for (;;) {
        uint32_t thr = (uint32_t)(ps * 16777216.0f);
        thr = thr < 0xFFFFFFu ? thr : 0xFFFFFFu;
        ent[s * kAS + lane] = (thr << 8) | (uint32_t)l;
        const float rest = (pl + ps) - 1.0f;
        const bool small = rest < 1.0f;  // l joins the small stack: pair it with a new large
        if (small ? nl == 0 : ns == 0) break;
        const int at = small ? K - nl : ns - 1;
        nl -= small ? 1 : 0;
        ns -= small ? 0 : 1;
        const int x = stk[at * 64 + lane];
        const float px = p[x * kAS + lane];
        s = small ? l : x;
        ps = small ? rest : px;
        l = small ? x : l;
        pl = small ? px : rest;
      }
      ent[l * kAS + lane] = 0xFFFFFF00u | (uint32_t)l;  // the carried index is left over
    }
    // leftovers keep their own index: what is still on either stack
    for (int i = 0; i < ns; ++i) {
      const int k = stk[i * 64 + lane];
      ent[k * kAS + lane] = 0xFFFFFF00u | (uint32_t)k;
    }
    for (int i = K - nl; i < K; ++i) {
      const int k = stk[i * 64 + lane];
      ent[k * kAS + lane] = 0xFFFFFF00u | (uint32_t)k;
    }
  }
  __syncthreads();
  // large vocabularies (many waves: store-throughput bound): word rows go out one row at a time,
  // lanes along k, so each store instruction writes 64 consecutive 16-B records (a lane per row
  // touches 64 rows K·16 B apart per store): 0.288 -> 0.244 ms at V = 180k, K = 100. Small ones
  // (few waves: latency bound) keep a lane per row: 0.049 vs 0.058 ms at V = 6.5k.
  const int nw = coal ? (int)(V - r0 < (int64_t)nrows ? (V - r0 > 0 ? V - r0 : 0) : nrows) : 0;
  if (!coal && word) {
    const uint32_t tb = __float_as_uint(tots[lane]);
    uint4* out = wrec + row * K;
#pragma unroll 4
    for (int k = 0; k < K; ++k) {
      const uint32_t e = ent[k * kAS + lane];
      out[k] = make_uint4(e, __float_as_uint(qr[k]), __float_as_uint(qr[e & 0xFFu]), tb);
    }
  }
#pragma unroll 2
  for (int r = 0; r < nw; ++r) {
    const float* qq = q + (r0 + r) * KS;
    const uint32_t tb = __float_as_uint(tots[r]);
    uint4* out = wrec + (r0 + r) * K;
    for (int k = lane; k < K; k += 64) {
      const uint32_t e = ent[k * kAS + r];
      out[k] = make_uint4(e, __float_as_uint(qq[k]), __float_as_uint(qq[e & 0xFFu]), tb);
    }
  }
  if (has) {
    if (word) {
      wsum[row] = tots[lane];
    } else {
      uint32_t* out = dalias + (row - V) * K;
#pragma unroll 4
      for (int k = 0; k < K; ++k) out[k] = ent[k * kAS + lane];
    }
  }
}

// ---- word proposal: level-1 CDF rows ----------------------------------------------------------------
// 16 lanes per word (4 words per wave): lane b sums bucket b's q values sequentially (the bucket's
// W = 8 or 16 topics, two or four 16-B loads of the q row: lanes along the row, coalesced), then
// takes C[b] = S_0 + … + S_b in order from its group's lanes and writes it: one 64-B row per word.
// Exactly spec.word_cdf.
template <int WB>
__global__ __launch_bounds__(256) void k_mh_cdf(const float* __restrict__ q, int64_t V, int K, int KS,
                                                float* __restrict__ wcdf) {
  const int lane = threadIdx.x & 63;
  const int bk = lane & 15;
  const int nb = (K + WB - 1) / WB;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r0 = wave * 4; r0 < V; r0 += nwaves * 4) {
    const int64_t row = r0 + (lane >> 4);
    const bool live = row < V;
    float sb = 0.f;
    if (live && bk < nb) {
      const float* qr = q + row * KS + bk * WB;
#pragma unroll
      for (int j4 = 0; j4 < WB / 4; ++j4) {
        const int k0 = bk * WB + 4 * j4;
        if (k0 < KS) {
          const float4 v = *reinterpret_cast<const float4*>(qr + 4 * j4);
          if (k0 + 0 < K) sb = sb + v.x;
          if (k0 + 1 < K) sb = sb + v.y;
          if (k0 + 2 < K) sb = sb + v.z;
          if (k0 + 3 < K) sb = sb + v.w;
        }
      }
    }
    float c = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float si = __shfl(sb, (lane & ~15) + i);
      if (i <= bk && i < nb) c = c + si;
    }
    if (live) wcdf[row * 16 + bk] = c;
  }
}

// ---- the sweep -----------------------------------------------------------------------------------
// LDS per block (one wave): (A, B) token-exclusion pairs and g per topic, then the u8 count cells
// [KS][64] and the chunk topics [lmax][64].
struct MHLds {
  float2* qfx;
  float* gk;
  uint8_t* cnt;
  uint8_t* zsl;
  float* c1s;  // level-1 CDF rows of the wave's 64 tokens, [64][kC1S] (after zsl; not with R5)
};
constexpr int kC1S = 20;  // c1 staging row stride (floats): 16-B aligned, rows 20 banks apart

// stage-B data of one token (issued one step ahead; none of it depends on the chain state)
template <int DM>
struct MHB {
  oni::U4 r;     // Philox block (pos, key, sweep, 2)
  int zo;        // sweep-start topic
  float qz;      // q[w, zo]
  uint4 rw;      // wp 0: word proposal record at j(r.x): {entry, q_j, q_alias, Σ_k q_k}
  float zw;      // wp > 0: Σ_k q[w, k] as the word CDF's total Z
  float qtw;     // wp > 0: q[w, tw] (stage C, from the bucket's q values)
  uint32_t ed;   // doc alias entry at j(r.z) (read for every chunk; used by multi-chunk docs)
  int32_t bzo;   // n_src[doc, zo]
  // stage C (issued at the end of the previous step, once that token has moved)
  int tw, td;    // word / doc proposals
  float qtd;     // q[w, td]
  int32_t btw, btd;  // n_src[doc, tw / td] (multi-chunk docs)
  // second doc move (DM = 2): Philox block (pos, key, sweep, 3) words z / w, its proposal and gathers
  // doc moves 2..DM: Philox2x32 words (proposal, acceptance), doc alias entry, proposal, gathers
  uint32_t r2z[DM > 1 ? DM - 1 : 1], r2w[DM > 1 ? DM - 1 : 1], ed2[DM > 1 ? DM - 1 : 1];
  int td2[DM > 1 ? DM - 1 : 1];
  float qtd2[DM > 1 ? DM - 1 : 1];
  int32_t btd2[DM > 1 ? DM - 1 : 1];
};

// Straight-line step: every lane issues the same loads (padding lanes on word 0, one-chunk docs
// on one common address for the doc tables) and every decision is a select, so no loaded value is
// merged at a control-flow join -- a merge there makes the compiler wait for every outstanding
// memory op (vmcnt(0)), which serialised the token pipeline.
// R5 (A/B, ONI_SAMPLER_AB & 32): round 5's level-1 rows (one lane per row, issued at the end of the
// step before their use, words two tokens ahead)
template <int MODE, int DM, int WP, bool R5 = false>
struct MHLane {
  // CDF word proposal: level-1 rows gathered four lanes per row (CO) and issued a whole step before
  // their use; words read four tokens ahead (WD; with the alias records they only feed stage B)
  static constexpr bool CO = !R5 && WP > 0;
  static constexpr bool WD = !R5;
  static constexpr int WB = WP > 0 ? WP : 1;
  const OniMH& m;
  const OniGibbs& a;
  MHLds L;
  int lane;
  int64_t off;
  int K, KS;
  bool multi;
  int lc;               // chunk length
  uint32_t pos0, key, sweep;
  uint32_t key2[DM > 1 ? DM - 1 : 1];  // per-sweep keys of doc moves 2..DM (Philox2x32 streams)
  const int32_t* brow;  // n_src row of the doc
  const uint32_t* drow; // dalias row of the doc (row 0 for one-chunk docs)
  uint32_t wa[2];       // stage A: token words (parity slots)
  uint32_t wb[2];       // WD: the words two tokens further ahead (parity slots)
  int64_t last;         // WD: SELL index of this lane's slot in the slice's last step
  int32_t pa[2];        // stage A: word-sorted slots (MODE 3/4)
  MHB<DM> b[2];             // stage B (parity slots)
  float c1[16];         // level-1 word CDF row of the token after next (gathered a step ahead of its stage B)
  float4 c1v[4];        // CO: this lane's quarter of rows 16 i + lane / 4 (i = 0..3), in flight
  float qb[WB];         // the proposed bucket's q values (stage B → stage C of one token)
  float ywd;            // the word draw's y = u·Z
  float base;           // C[bucket − 1] (gathered)
  int bk;               // the bucket
  int32_t* red;         // LDS: per-topic count deltas of the wave
  int nchg;
  Pend<MODE> pend;

  __device__ __forceinline__ MHLane(const OniMH& m_) : m(m_), a(m_.g) {}

  __device__ __forceinline__ int cell(int k) const { return (int)L.cnt[k * 64 + lane]; }
  __device__ __forceinline__ void cell_set(int k, int v) { L.cnt[k * 64 + lane] = (uint8_t)v; }
  // n_dk^¬ + α from a count cell c and the sweep-start count bk
  __device__ __forceinline__ float aw(int c, int32_t bk) const {
    return (float)(multi ? bk + c - kMHBias : c) + a.alpha;
  }
  __device__ __forceinline__ bool alias_keeps(uint32_t r, uint32_t e) const {
    return ((r * (uint32_t)K) >> 8) < (e >> 8);
  }
  __device__ __forceinline__ int alias_draw(uint32_t r, uint32_t e) const {
    const int j = (int)__umulhi(r, (uint32_t)K);
    return alias_resolve(j, (r * (uint32_t)K) >> 8, e);
  }
  // one-chunk documents: a random other token's current topic, or a uniform topic
  __device__ __forceinline__ int single_pick(uint32_t r, int s) const {
    const float nd = (float)(lc - 1);
    const float y = oni::u01(r) * (nd + m.kalpha);
    int pp = (int)y;
    pp += pp >= s ? 1 : 0;
    pp = pp < lc ? pp : 0;
    const int tz = (int)L.zsl[pp * 64 + lane];
    int tu = (int)((y - nd) * m.inv_alpha);
    tu = tu < K - 1 ? tu : K - 1;
    return y < nd ? tz : tu;
  }

  // level-1 word CDF row of word w (a stage ahead of its stage B: its bucket gather depends on it)
  // CO: the 64 rows are gathered four lanes per row (lane l loads quarter l % 4 of row 16 i + l / 4
  // in load i): each load touches 16 lines instead of 64, a quarter of the address-unit work of one
  // row per lane (the TA unit was the busiest one of this kernel, profiles/r6/mh_pmc/). The rows are
  // turned back to one per lane through LDS when they are used (land_c1).
  __device__ __forceinline__ void load_c1(uint32_t w) {
    if constexpr (WP == 0) return;
    if constexpr (CO) {
      const int wc = (int)(w == oni::kPadWord ? 0u : w);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t wr = (uint32_t)__shfl(wc, 16 * i + (lane >> 2));
        c1v[i] = reinterpret_cast<const float4*>(m.wcdf)[(int64_t)wr * 4 + (lane & 3)];
      }
      return;
    }
    const float4* r = reinterpret_cast<const float4*>(m.wcdf) + (int64_t)(w == oni::kPadWord ? 0u : w) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 v = r[i];
      c1[4 * i] = v.x;
      c1[4 * i + 1] = v.y;
      c1[4 * i + 2] = v.z;
      c1[4 * i + 3] = v.w;
    }
  }

  // CO: the quarters in flight to LDS, then this lane's own row back (one wave: its LDS accesses
  // run in order; the fences keep the compiler from reordering them)
  __device__ __forceinline__ void land_c1() {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<float4*>(L.c1s + (16 * i + (lane >> 2)) * kC1S + 4 * (lane & 3)) = c1v[i];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 v = *reinterpret_cast<const float4*>(L.c1s + lane * kC1S + 4 * i);
      c1[4 * i] = v.x;
      c1[4 * i + 1] = v.y;
      c1[4 * i + 2] = v.z;
      c1[4 * i + 3] = v.w;
    }
    asm volatile("" ::: "memory");
  }

  // stage B of the token at step s (word w): Philox block, then the state-free gathers
  __device__ __forceinline__ void issue_b(int P, int s, uint32_t w) {
    if constexpr (CO) land_c1();
    MHB<DM>& x = b[P];
    const uint32_t wc = w == oni::kPadWord ? 0u : w;
    x.r = oni::philox10(oni::U4{pos0 + (uint32_t)s, key, sweep, 2u}, a.seed0, a.seed1);
    const int z0 = (int)L.zsl[s * 64 + lane];
    x.zo = z0 < K - 1 ? z0 : K - 1;  // padding slots hold 0; clamp anyway: an LDS index
    x.qz = a.q[wc * (uint32_t)KS + (uint32_t)x.zo];
    if constexpr (WP == 0) {
      x.rw = m.walias[wc * (uint32_t)K + __umulhi(x.r.x, (uint32_t)K)];
    } else {
    // word proposal, level 1: y = u·Z, bucket = #{i : C[i] ≤ y} (capped; a branch-free binary search
    // over the monotone row), residual y − C[b − 1]
      const int nb = (K + WB - 1) / WB;
      x.zw = c1[15];
      ywd = oni::u01(x.r.x) * c1[15];
      const int nbk = count_le<16>(c1, 0.f, ywd);
      bk = nbk < nb - 1 ? nbk : nb - 1;
      // C[b − 1] selected from the registers (a gather here measured 14 % slower: one more load in
      // the token pipeline's in-order vmcnt)
      base = 0.f;
#pragma unroll
      for (int i = 0; i < 15; ++i) base = i == bk - 1 ? c1[i] : base;
      // level 2: the bucket's q values (a float4 past the row's KS padding is not read)
      const float* qr = a.q + (int64_t)wc * KS + bk * WB;
#pragma unroll
      for (int j4 = 0; j4 < WB / 4; ++j4) {
        const bool in = bk * WB + 4 * j4 < KS;
        const float4 v = *reinterpret_cast<const float4*>(in ? qr + 4 * j4 : a.q);
        qb[4 * j4] = in ? v.x : 0.f;
        qb[4 * j4 + 1] = in ? v.y : 0.f;
        qb[4 * j4 + 2] = in ? v.z : 0.f;
        qb[4 * j4 + 3] = in ? v.w : 0.f;
      }
    }
    // one-chunk docs read one common address (they use neither value): no scattered lines
    x.ed = drow[multi ? __umulhi(x.r.z, (uint32_t)K) : 0u];
    x.bzo = brow[multi ? x.zo : 0];
#pragma unroll
    for (int c = 0; c < DM - 1; ++c) {
      uint32_t c0 = pos0 + (uint32_t)s, c1 = key;
      oni::philox2x32_10(c0, c1, key2[c]);
      x.r2z[c] = c0;
      x.r2w[c] = c1;
      x.ed2[c] = drow[multi ? __umulhi(c0, (uint32_t)K) : 0u];
    }
  }

  // stage C of the token at step s: its proposals (the one-chunk doc proposal reads the chunk's
  // current topics, so this runs after the previous token has moved) and their gathers
  __device__ __forceinline__ void issue_c(int P, int s, uint32_t w) {
    MHB<DM>& x = b[P];
    const uint32_t qo = (w == oni::kPadWord ? 0u : w) * (uint32_t)KS;
    if constexpr (WP == 0) {
      x.tw = alias_draw(x.r.x, x.rw.x);
    } else {
      // word proposal, level 2: running f32 sum of the bucket's q values from 0 (spec.word_cdf_draw).
      // Topics past K hold q = 0 (k_apply) and the loads past KS were zeroed: their running sums
      // repeat the last real one, so counting them changes nothing after the cap.
      const float y2 = ywd - (bk > 0 ? base : 0.f);
      float cum[WB];
      float run = 0.f;
#pragma unroll
      for (int j = 0; j < WB; ++j) {
        run = run + qb[j];
        cum[j] = run;
      }
      const int cnt = count_le<WB>(cum, 0.f, y2);
      const int rem = K - bk * WB;
      const int last = (rem < WB ? rem : WB) - 1;
      const int tin = cnt < last ? cnt : last;
      float qt = qb[0];
#pragma unroll
      for (int j = 1; j < WB; ++j) qt = j == tin ? qb[j] : qt;
      x.tw = bk * WB + tin;
      x.qtw = qt;
    }
    const int tdm = alias_draw(x.r.z, x.ed);
    const int tds = single_pick(x.r.z, s);
    x.td = multi ? tdm : tds;
    x.qtd = a.q[qo + (uint32_t)x.td];
    x.btw = brow[multi ? x.tw : 0];
    x.btd = brow[multi ? x.td : 0];
    // the later doc moves' proposals are state-free too (the chunk's other topics do not move
    // while this token does): prefetched with the first
#pragma unroll
    for (int c = 0; c < DM - 1; ++c) {
      const int t2m = alias_draw(x.r2z[c], x.ed2[c]);
      const int t2s = single_pick(x.r2z[c], s);
      x.td2[c] = multi ? t2m : t2s;
      x.qtd2[c] = a.q[qo + (uint32_t)x.td2[c]];
      x.btd2[c] = brow[multi ? x.td2[c] : 0];
    }
  }

  // one token: word move, doc move(s), bookkeeping. The next token's prefetches are issued before
  // this token's math, its stage C after it (the issue order is the wait order: one in-order vmcnt;
  // pinned by compiler fences).
  template <int P, bool LOAD_A, bool LOAD_B>
  __device__ __forceinline__ void step(int s) {
    constexpr int NX = 1 - P;
    const int64_t idx = off + (int64_t)s * 64 + lane;
    const uint32_t w = wa[P];
    const int32_t pw = pa[P];
    const bool act = w != oni::kPadWord;
    const MHB<DM>& x = b[P];
    const int zo = x.zo;
    cell_set(zo, cell(zo) - (act ? 1 : 0));  // the token leaves its topic: every count below is n^¬
    asm volatile("" ::: "memory");
    if constexpr (LOAD_B) issue_b(NX, s + 1, wa[NX]);
    asm volatile("" ::: "memory");
    if constexpr (WD) {
      // the level-1 row of token s + 2 now (its word came two steps ago), used a step from now
      if constexpr (LOAD_B) load_c1(wb[P]);
      asm volatile("" ::: "memory");
      wa[P] = wb[P];
      // word of token s + 4 (clamped to the slice: past its end nothing uses it)
      const int64_t i4 = idx + 256;
      wb[P] = a.tok_word[i4 < last ? i4 : last];
      if constexpr (LOAD_A && (MODE == 3 || MODE == 4)) pa[P] = a.wpos[idx + 128];
    } else if constexpr (LOAD_A) {
      wa[P] = a.tok_word[idx + 128];
      if constexpr (MODE == 3 || MODE == 4) pa[P] = a.wpos[idx + 128];
    } else {
      wa[P] = oni::kPadWord;
    }
    asm volatile("" ::: "memory");
    pend.flush(a, KS);
    asm volatile("" ::: "memory");
    const int tw = x.tw, td = x.td;
    float qtw, zw;
    if constexpr (WP == 0) {
      qtw = __uint_as_float(alias_keeps(x.r.x, x.rw.x) ? x.rw.y : x.rw.z);
      zw = __uint_as_float(x.rw.w);
    } else {
      qtw = x.qtw;
      zw = x.zw;
    }
    const float qtd = x.qtd;
    const int32_t btw = x.btw, btd = x.btd;
    const float2 ab = L.qfx[zo];
    const float qe = fmaf(x.qz, ab.x, -ab.y);
    const float azo = aw(cell(zo), x.bzo);
    const float atw = aw(cell(tw), btw);
    const float atd = aw(cell(td), btd);
    // word move (from zo): ratio a_t Z_zo / (a_zo Z_t), Z_t = (Z_zo − (q_zo − q'_zo)) + (1 − q_t) g_t
    const float d = x.qz - qe;
    const float zt = (zw - d) + ((1.0f - qtw) * L.gk[tw]);
    const bool accw = (tw != zo) & (oni::u01(x.r.y) * (azo * zt) < atw * zw);
    int sc = accw ? tw : zo;
    float qs = accw ? qtw : qe;
    float as = accw ? atw : azo;
    int32_t bs = accw ? btw : x.bzo;
    // doc moves: one-chunk docs ratio q'_t / q'_s; multi-chunk docs (a_t q'_t bn_s) / (a_s q'_s bn_t),
    // bn = n_src without the token + α; from s ≠ zo a draw of zo is a no-op w.p. 1/(b_zo + α)
#pragma unroll
    for (int c = 0; c < DM; ++c) {
      uint32_t r3 = x.r.w;
      int t = td;
      float qt = td == zo ? qe : qtd;
      int32_t bt = btd;
      float at = atd;
      if constexpr (DM > 1) {
        if (c > 0) {
          r3 = x.r2w[c - 1];
          t = x.td2[c - 1];
          qt = t == zo ? qe : x.qtd2[c - 1];
          bt = x.btd2[c - 1];
          at = aw(cell(t), bt);
        }
      }
      const float u = oni::u01(r3);
      const float bnt = (float)(bt - (t == zo ? 1 : 0)) + a.alpha;
      const float bns = (float)(bs - (sc == zo ? 1 : 0)) + a.alpha;
      const float num = (at * qt) * bns;
      const float den = (as * qs) * bnt;
      const float bz = (float)bt + a.alpha;
      const bool sw = t == zo && sc != zo;
      const bool ok_sw = (u * bz < bnt) & ((u * den) * bz < num * bnt);
      const bool ok_m = sw ? ok_sw : (u * den < num);
      const bool ok_s = u * qs < qt;
      const bool ok = (multi ? ok_m : ok_s) & (t != sc);
      sc = ok ? t : sc;
      qs = ok ? qt : qs;
      as = ok ? at : as;
      bs = ok ? bt : bs;
    }
    const bool changed = act & (sc != zo);
    cell_set(sc, cell(sc) + (act ? 1 : 0));
    L.zsl[s * 64 + lane] = (uint8_t)sc;
    nchg += changed ? 1 : 0;
    pend.note(idx, zo, sc, pw, w);
    pend.on = changed;
    if (changed) {
      atomicAdd(&red[zo], -1);
      atomicAdd(&red[sc], 1);
    }
    if constexpr (MODE == 2) {
      const uint64_t msk = __ballot(changed);
      if (lane == 0) {
        pend.m = msk;
        pend.mi = (off + (int64_t)s * 64) / 64;
      }
    }
    asm volatile("" ::: "memory");
    if constexpr (LOAD_B) {
      if constexpr (!WD) load_c1(wa[P]);  // the token after next (issued before stage C: its wait must not cover C)
      asm volatile("" ::: "memory");
      issue_c(NX, s + 1, wa[NX]);
    }
  }
};

// segmented (same doc, consecutive lanes) suffix sum: the run's first lane gets the run total
__device__ __forceinline__ int run_sum(int v, int c, int next) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_down(v, o);
    if (c + o < next) v += t;
  }
  return v;
}

// Epilogue: one-chunk docs store their row; multi-chunk docs add their deltas (summed over the
// wave's consecutive chunks of the same doc first). The per-topic deltas were counted in LDS
// (`red`, one ds_add per move) and go to one dnk replica.
__device__ __forceinline__ void mh_epilogue(const OniMH& m, const MHLds& L, int KS, int lane, int doc, bool live,
                                            bool multi, const int32_t* red) {
  const OniGibbs& a = m.g;
  const int prev_doc = __shfl_up(doc, 1);
  const bool head = lane == 0 || prev_doc != doc;
  const uint64_t heads = __ballot(head);
  const uint64_t above = lane < 63 ? heads & (~0ull << (lane + 1)) : 0ull;
  const int next = above ? __ffsll((unsigned long long)above) - 1 : 64;
  const bool any_multi = __ballot(live && multi) != 0ull;
  int32_t* dst = a.ndk_dst + (int64_t)(live ? doc : 0) * KS;
#pragma unroll 2
  for (int k0 = 0; k0 < KS; k0 += 4) {
    int c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = (int)L.cnt[(k0 + i) * 64 + lane];
    if (live && !multi) *reinterpret_cast<int4*>(dst + k0) = make_int4(c[0], c[1], c[2], c[3]);
    if (any_multi) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int d = live && multi ? c[i] - kMHBias : 0;
        if (__ballot(d != 0)) {
          const int sm = run_sum(d, lane, next);
          if (live && multi && head && sm) atomicAdd(dst + k0 + i, sm);
        }
      }
    }
  }
  __syncthreads();
  for (int k = lane; k < KS; k += 64) {
    const int v = red[k];
    if (v) atomicAdd(&a.dnk[(int)(blockIdx.x & (unsigned)(a.nk_rep - 1)) * KS + k], v);
  }
}

// the slice's topics into LDS: the SELL slice is len rows of 64 bytes, exactly the [s][lane] layout
__device__ __forceinline__ void load_slice_topics(const OniGibbs& a, uint8_t* zsl, int64_t off, int len) {
  const uint4* src = reinterpret_cast<const uint4*>(a.tok_z + off);
  uint4* dst = reinterpret_cast<uint4*>(zsl);
  for (int i = threadIdx.x; i < len * 4; i += 64) dst[i] = src[i];
}

__device__ __forceinline__ MHLds mh_lds(unsigned char* smem, int KS) {
  MHLds L;
  L.qfx = reinterpret_cast<float2*>(smem);
  L.gk = reinterpret_cast<float*>(smem + (size_t)KS * sizeof(float2));
  L.cnt = smem + (size_t)KS * (sizeof(float2) + sizeof(float) + sizeof(int32_t));
  L.zsl = L.cnt + (size_t)KS * 64;
  return L;
}

template <int MODE, int DM, int WP, bool R5 = false>
__global__ __launch_bounds__(64) void k_gibbs_mh(const OniMH m) {
  extern __shared__ __align__(16) unsigned char smem_mh[];
  const OniGibbs& a = m.g;
  const int KS = a.KS;
  MHLane<MODE, DM, WP, R5> x(m);
  x.L = mh_lds(smem_mh, KS);
  x.L.c1s = reinterpret_cast<float*>(x.L.zsl + (size_t)m.lmax * 64);
  int32_t* red = reinterpret_cast<int32_t*>(smem_mh + (size_t)KS * (sizeof(float2) + sizeof(float)));
  x.red = red;
  const int lane = threadIdx.x;
  x.lane = lane;
  x.K = a.K;
  x.KS = KS;
  for (int k = lane; k < KS; k += 64) {
    x.L.qfx[k] = make_float2(a.qfix[k], a.qfix[KS + k]);
    x.L.gk[k] = m.mh_g[k];
    red[k] = 0;
  }
  const int64_t slice = blockIdx.x;
  const int64_t chunk = slice * 64 + lane;
  const int doc = a.chunk_doc[chunk];
  const bool live = doc >= 0;
  x.multi = live && a.chunk_multi[chunk] != 0;
  x.drow = m.dalias + (int64_t)(x.multi ? m.chunk_dslot[chunk] : 0) * a.K;
  x.lc = live ? m.chunk_len[chunk] : 0;
  x.pos0 = live ? (uint32_t)a.chunk_pos0[chunk] : 0u;
  x.key = live ? a.chunk_key[chunk] : 0u;
  x.sweep = *a.sweep_ctr;
#pragma unroll
  for (int c = 0; c < DM - 1; ++c)
    x.key2[c] = oni::philox10(oni::U4{x.sweep, 3u + (uint32_t)c, 0x4D48u, 0u}, a.seed0, a.seed1).x;
  const int32_t* own = a.ndk_src + (int64_t)(live ? doc : 0) * KS;
  // multi-chunk docs read their sweep-start row; one-chunk docs never use it and read one common
  // address instead (row 0, index 0), so their lanes add no scattered lines to the gathers
  x.brow = x.multi ? own : a.ndk_src;
  x.nchg = 0;
  const int len = a.slice_len[slice];
  x.off = a.slice_off[slice];
  // count cells: n (one-chunk docs, ≤ 127) or the bias (multi-chunk docs); chunk topics
  load_slice_topics(a, x.L.zsl, x.off, len);
#pragma unroll 5
  for (int k = 0; k < KS; k += 4) {
    int4 v = make_int4(0, 0, 0, 0);
    if (live) v = x.multi ? make_int4(kMHBias, kMHBias, kMHBias, kMHBias) : *reinterpret_cast<const int4*>(own + k);
    x.L.cnt[k * 64 + lane] = (uint8_t)v.x;
    x.L.cnt[(k + 1) * 64 + lane] = (uint8_t)v.y;
    x.L.cnt[(k + 2) * 64 + lane] = (uint8_t)v.z;
    x.L.cnt[(k + 3) * 64 + lane] = (uint8_t)v.w;
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    x.wa[t] = len > t ? a.tok_word[x.off + t * 64 + lane] : oni::kPadWord;
    x.pa[t] = ((MODE == 3 || MODE == 4) && len > t) ? a.wpos[x.off + t * 64 + lane] : 0;
    x.wb[t] = len > t + 2 ? a.tok_word[x.off + (t + 2) * 64 + lane] : oni::kPadWord;
  }
  x.last = x.off + (int64_t)(len > 0 ? len - 1 : 0) * 64 + lane;
  x.load_c1(x.wa[0]);
  x.issue_b(0, 0, x.wa[0]);
  x.load_c1(x.wa[1]);
  x.issue_c(0, 0, x.wa[0]);
  int s = 0;
  for (; s + 3 < len; s += 2) {
    x.template step<0, true, true>(s);
    x.template step<1, true, true>(s + 1);
  }
  for (; s < len; s += 2) {  // the last ≤ 3 steps
    if (s + 2 < len) x.template step<0, true, true>(s);
    else if (s + 1 < len) x.template step<0, false, true>(s);
    else x.template step<0, false, false>(s);
    if (s + 2 < len) x.template step<1, false, true>(s + 1);
    else if (s + 1 < len) x.template step<1, false, false>(s + 1);
  }
  x.pend.flush(a, KS);
  if (a.chg_count) add_wave_count(a.chg_count, x.nchg);
  __syncthreads();
  mh_epilogue(m, x.L, KS, lane, doc, live, x.multi, red);
}

// init pass (one-lane units, any K): z = ⌊r·K / 2^32⌋ with r the generic init's draw (stream 0,
// one Philox block per 4 positions) -- the same topics as spec.gibbs_pass(init=True)
__global__ __launch_bounds__(64) void k_gibbs_mh_init(const OniMH m) {
  extern __shared__ __align__(16) unsigned char smem_mh[];
  const OniGibbs& a = m.g;
  const int KS = a.KS;
  MHLds L = mh_lds(smem_mh, KS);
  int32_t* red = reinterpret_cast<int32_t*>(smem_mh + (size_t)KS * (sizeof(float2) + sizeof(float)));
  const int lane = threadIdx.x;
  const int64_t slice = blockIdx.x;
  const int64_t chunk = slice * 64 + lane;
  const int doc = a.chunk_doc[chunk];
  const bool live = doc >= 0;
  const bool multi = live && a.chunk_multi[chunk] != 0;
  const int lc = live ? m.chunk_len[chunk] : 0;
  const uint32_t pos0 = live ? (uint32_t)a.chunk_pos0[chunk] : 0u;
  const uint32_t key = live ? a.chunk_key[chunk] : 0u;
  const int64_t off = a.slice_off[slice];
  for (int k = 0; k < KS; ++k) L.cnt[k * 64 + lane] = (uint8_t)(live && multi ? kMHBias : 0);
  for (int k = lane; k < KS; k += 64) red[k] = 0;
  __syncthreads();
  for (int s = 0; s < lc; ++s) {
    const uint32_t pos = pos0 + (uint32_t)s;
    uint32_t rr;
    if (a.flags & 8) {
      rr = oni::mix32(a.tok_word[off + (int64_t)s * 64 + lane]);
    } else {
      const oni::U4 r = oni::philox10(oni::U4{pos >> 2, key, 0u, 0u}, a.seed0, a.seed1);
      rr = oni::pick4(r, pos & 3u);
    }
    const int z = (int)(((uint64_t)rr * (uint32_t)a.K) >> 32);
    L.cnt[z * 64 + lane] = (uint8_t)((int)L.cnt[z * 64 + lane] + 1);
    atomicAdd(&red[z], 1);
    a.tok_z[off + (int64_t)s * 64 + lane] = (uint8_t)z;
  }
  __syncthreads();
  mh_epilogue(m, L, KS, lane, doc, live, multi, red);
}

}  // namespace

static size_t mh_lds_bytes(int KS, int lmax, bool co) {
  return (size_t)KS * (sizeof(float2) + sizeof(float) + sizeof(int32_t)) + (size_t)KS * 64 + (size_t)lmax * 64 +
         (co ? (size_t)64 * kC1S * sizeof(float) : 0);
}

// Per-sweep MH tables. Word proposal: alias records (walias + wsum, k_mh_alias over the V word rows)
// or the level-1 CDF rows (wcdf, k_mh_cdf); exactly one of the two. Then the alias rows of the n_long
// multi-chunk documents and g (k_mh_alias, document rows).
ONI_API int oni_mh_tables(const float* q, int64_t V, int K, int KS, const int32_t* ndk, const int32_t* rows,
                          int64_t n_long, float alpha, uint4* walias, float* wsum, float* wcdf, uint32_t* dalias,
                          const int32_t* nk, float vbeta, float* g, hipStream_t s) {
  if (K < 1 || K > 255 || K > KS || KS % 4 || V < 0 || n_long < 0) return (int)hipErrorInvalidValue;
  if ((walias == nullptr) == (wcdf == nullptr) || (walias != nullptr && wsum == nullptr))
    return (int)hipErrorInvalidValue;
  int64_t Vw = V;
  if (wcdf != nullptr) {
    if (V > 0) {
      const unsigned cgrid = oni::grid_for((V + 3) / 4 * 64, 256, 8192);
      if (K <= 128) k_mh_cdf<8><<<cgrid, 256, 0, s>>>(q, V, K, KS, wcdf);
      else k_mh_cdf<16><<<cgrid, 256, 0, s>>>(q, V, K, KS, wcdf);
    }
    Vw = 0;
  }
  const int64_t nrows = Vw + n_long;
  const unsigned grid = (unsigned)((nrows + 63) / 64 > 0 ? (nrows + 63) / 64 : 1);
  const size_t lds = (size_t)K * kAS * sizeof(float) + 64 * sizeof(float) + (size_t)K * 64;
  k_mh_alias<<<grid, 64, lds, s>>>(q, Vw, K, KS, ndk, rows, n_long, alpha, walias, wsum, dalias, nk, vbeta, g,
                                   Vw >= 65536);
  return (int)hipGetLastError();
}

ONI_API int oni_gibbs_mh_launch(const OniMH* m, int init, int mode, hipStream_t s) {
  const OniGibbs& a = m->g;
  if (a.K < 1 || a.K > 255 || a.K > a.KS || a.KS % 4 || a.KS > 256 || mode < 0 || mode > 4) return (int)hipErrorInvalidValue;
  if (a.nk_rep < 1 || (a.nk_rep & (a.nk_rep - 1))) return (int)hipErrorInvalidValue;
  if (m->lmax < 1 || m->lmax > 127 || !m->chunk_len) return (int)hipErrorInvalidValue;
  if (a.n_slices < 1) return 0;
  const unsigned grid = (unsigned)a.n_slices;
  if (init) {
    k_gibbs_mh_init<<<grid, 64, mh_lds_bytes(a.KS, m->lmax, false), s>>>(*m);
    return (int)hipGetLastError();
  }
  if (!a.qfix || !m->mh_g || !m->chunk_dslot) return (int)hipErrorInvalidValue;
  if (m->wp == 0 ? (!m->walias || !m->wsum) : (!m->wcdf || m->wp != (a.K <= 128 ? 8 : 16)))
    return (int)hipErrorInvalidValue;
  if (m->doc_moves < 1 || m->doc_moves > 4) return (int)hipErrorInvalidValue;
  if (mode == 2 && !a.chg_mask) return (int)hipErrorInvalidValue;
  if (mode == 3 && (!a.wpos || !a.z_w)) return (int)hipErrorInvalidValue;
  if (mode == 4 && (!a.wpos || !a.zz_w || !a.chg_mask)) return (int)hipErrorInvalidValue;
  const bool r5 = (a.flags & 512) != 0;  // A/B: round 5's level-1 row gathers
  const size_t lds = mh_lds_bytes(a.KS, m->lmax, m->wp > 0 && !r5);
  if (r5 && m->doc_moves == 2 && (m->wp == 8 || m->wp == 0) && (mode == 0 || mode == 4)) {
    if (m->wp == 8) {
      if (mode == 0) k_gibbs_mh<0, 2, 8, true><<<grid, 64, lds, s>>>(*m);
      else k_gibbs_mh<4, 2, 8, true><<<grid, 64, lds, s>>>(*m);
    } else {
      if (mode == 0) k_gibbs_mh<0, 2, 0, true><<<grid, 64, lds, s>>>(*m);
      else k_gibbs_mh<4, 2, 0, true><<<grid, 64, lds, s>>>(*m);
    }
    return (int)hipGetLastError();
  }
#define ONI_MH(md, dm)                                                  \
  do {                                                                  \
    if (m->wp == 0) k_gibbs_mh<md, dm, 0><<<grid, 64, lds, s>>>(*m);    \
    else if (m->wp == 8) k_gibbs_mh<md, dm, 8><<<grid, 64, lds, s>>>(*m); \
    else k_gibbs_mh<md, dm, 16><<<grid, 64, lds, s>>>(*m);              \
  } while (0)
  switch (m->doc_moves * 8 + mode) {
#define ONI_MH_CASES(dm) \
    case dm * 8 + 0: ONI_MH(0, dm); break; \
    case dm * 8 + 1: ONI_MH(1, dm); break; \
    case dm * 8 + 2: ONI_MH(2, dm); break; \
    case dm * 8 + 3: ONI_MH(3, dm); break; \
    case dm * 8 + 4: ONI_MH(4, dm); break;
    ONI_MH_CASES(1) ONI_MH_CASES(2) ONI_MH_CASES(3) ONI_MH_CASES(4)
#undef ONI_MH_CASES
    default: return (int)hipErrorInvalidValue;
  }
#undef ONI_MH
  return (int)hipGetLastError();
}

ONI_API int oni_mh_sizeof_args() { return (int)sizeof(OniMH); }
