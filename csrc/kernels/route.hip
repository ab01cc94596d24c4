// Data-parallel token routing: pack every token for its document's owner rank.
//
// The reference shipped whole corpus files to the MPI ranks of oni-lda-c ([U-H]). Here each rank
// featurizes its own events and every token (doc key, word id[, weight]) must reach the rank that
// owns its document before the corpus build. route_pack turns "owner of every local document" into
// the all-to-all send buffer with one stable partition by owner, written straight into the packed
// int32 columns (8 B per token, 12 B with weights, instead of three int64 columns): a per-tile owner
// histogram, one scan over the (owner, tile) counts, and a scatter pass whose in-tile ranks come from
// wave ballots (no radix sort, no separate gather). ``order`` (slot → token) is what the way back
// (oni355.pipeline.common.return_to_origin) scatters through. The same partition groups the local
// documents by owner (the key lists sent ahead of the tokens), and two small kernels do the document
// placement bookkeeping of pipeline.common.place_docs (candidate counts, hash-bucket loads, owner of
// every document) in one pass each instead of a dozen torch ops.
#include <hipcub/hipcub.hpp>

#include "oni_common.h"

namespace {

constexpr int kB = 256;
inline unsigned nblk(int64_t n) { return (unsigned)((n + kB - 1) / kB > 0 ? (n + kB - 1) / kB : 1); }

struct Arena {
  char* base;
  size_t used = 0;
  template <class T>
  T* take(size_t n) {
    used = (used + 255) & ~size_t(255);
    T* p = base ? reinterpret_cast<T*>(base + used) : nullptr;
    used += n * sizeof(T);
    return p;
  }
};

// Owner side of the id routing: row j of the received buffer came from the source rank whose
// segment [seg[s], seg[s+1]) holds it; its column 0 indexes that source's key list, whose
// dictionary ids start at kid + koff[s]. Writes the token's owner-local doc id, word and weight.
__global__ void k_route_unpack(const int32_t* __restrict__ recv, int64_t n, int C, const int64_t* __restrict__ seg,
                               const int64_t* __restrict__ koff, int W, const int32_t* __restrict__ kid,
                               int32_t* __restrict__ doc, int32_t* __restrict__ word, int32_t* __restrict__ wt) {
  __shared__ int64_t s_seg[257];
  __shared__ int64_t s_koff[256];
  for (int i = threadIdx.x; i <= W; i += kB) s_seg[i] = seg[i];
  for (int i = threadIdx.x; i < W; i += kB) s_koff[i] = koff[i];
  __syncthreads();
  const int64_t j = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (j >= n) return;
  int lo = 0, hi = W - 1;  // last source s with seg[s] <= j
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s_seg[mid] <= j) lo = mid;
    else hi = mid - 1;
  }
  doc[j] = kid[s_koff[lo] + recv[j * C]];
  word[j] = recv[j * C + 1];
  if (wt) wt[j] = C == 3 ? recv[j * C + 2] : 1;
}

// ---- stable partition by owner -----------------------------------------------------------------
// Items are processed in tiles of kTile (one block): round r of a block covers kPT consecutive
// items, one per thread, so (tile, round, wave, lane) is item order and the slot of an item is
//   off[owner][tile] + Σ_{earlier rounds} + Σ_{earlier waves of this round} + rank in its wave.
// Ranks in a wave come from peeling the distinct owners present with ballots (≤ 64 iterations,
// usually W). Owners outside [0, W) are clamped (memory safety; the callers produce valid owners).
constexpr int kPT = 256;
constexpr int kPR = 8;
constexpr int kTile = kPT * kPR;
constexpr int kPW = kPT / 64;

struct PartIn {
  const int32_t* owner_of_id;  // owner of item i is owner_of_id[ids ? ids[i] : i]
  const int32_t* ids;
  int64_t n;
  int W;
  int nb;  // tiles
};

__device__ __forceinline__ int item_owner(const PartIn& p, int64_t i) {
  int o = p.owner_of_id[p.ids ? p.ids[i] : i];
  return o < 0 ? 0 : (o >= p.W ? p.W - 1 : o);
}

__device__ __forceinline__ int lanes_below(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__global__ __launch_bounds__(kPT) void k_part_hist(PartIn p, int32_t* __restrict__ blkcnt,
                                                   unsigned long long* __restrict__ counts) {
  __shared__ int h[256];
  for (int o = threadIdx.x; o < p.W; o += kPT) h[o] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * kTile;
  for (int r = 0; r < kPR; ++r) {
    const int64_t i = t0 + (int64_t)r * kPT + threadIdx.x;
    const bool valid = i < p.n;
    const int own = valid ? item_owner(p, i) : -1;
    uint64_t active = __ballot(valid);
    while (active) {
      const int leader = __ffsll((unsigned long long)active) - 1;
      const int o = __builtin_amdgcn_readlane(own, leader);
      const uint64_t m = __ballot(own == o);
      if (oni::lane_id() == leader) atomicAdd(&h[o], __popcll(m));
      active &= ~m;
    }
  }
  __syncthreads();
  for (int o = threadIdx.x; o < p.W; o += kPT) {
    blkcnt[(int64_t)o * p.nb + blockIdx.x] = h[o];
    if (h[o]) atomicAdd(&counts[o], (unsigned long long)h[o]);
  }
}

// what a partition writes for item i at slot `slot` of the owner-grouped output
struct EmitPart {
  int32_t* order;          // slot → item
  int32_t* rank;           // item → slot - start of its owner's group (optional)
  const int64_t* keys;     // optional: keys_out[slot] = u32 bits of keys[i]
  int32_t* keys_out;
  const int32_t* off;
  int nb;
  __device__ void operator()(int64_t i, int slot, int own) const {
    order[slot] = (int32_t)i;
    if (rank) rank[i] = slot - off[(int64_t)own * nb];
    if (keys_out) keys_out[slot] = (int32_t)(uint32_t)(uint64_t)keys[i];
  }
};

// the routing send row: column 0 the doc key's u32 bits, or with DOCVAL doc_val[ids[i]] (the
// document's position in the key list sent to its owner); then word[, weight]
template <int C, bool DOCVAL>
struct EmitRoute {
  int32_t* order;
  int32_t* send;
  const int64_t* keys;
  const int32_t* ids;
  const int32_t* doc_val;
  const int32_t* word;
  const int32_t* weight;
  __device__ void operator()(int64_t i, int slot, int) const {
    order[slot] = (int32_t)i;
    int32_t* row = send + (int64_t)slot * C;
    if constexpr (DOCVAL) row[0] = doc_val[ids[i]];
    else row[0] = (int32_t)(uint32_t)(uint64_t)keys[i];
    row[1] = word[i];
    if constexpr (C == 3) row[2] = weight[i];
  }
};

template <class Emit>
__global__ __launch_bounds__(kPT) void k_part_scatter(PartIn p, const int32_t* __restrict__ off, Emit emit) {
  __shared__ int base[256];
  __shared__ int wc[kPW][256];
  const int lane = oni::lane_id(), wv = threadIdx.x >> 6;
  for (int o = threadIdx.x; o < p.W; o += kPT) {
    base[o] = off[(int64_t)o * p.nb + blockIdx.x];
    for (int w = 0; w < kPW; ++w) wc[w][o] = 0;
  }
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * kTile;
  for (int r = 0; r < kPR; ++r) {
    const int64_t i = t0 + (int64_t)r * kPT + threadIdx.x;
    const bool valid = i < p.n;
    const int own = valid ? item_owner(p, i) : -1;
    uint64_t active = __ballot(valid);
    int rank = 0;
    while (active) {
      const int leader = __ffsll((unsigned long long)active) - 1;
      const int o = __builtin_amdgcn_readlane(own, leader);
      const uint64_t m = __ballot(own == o);
      if (own == o) rank = lanes_below(m);
      if (lane == leader) wc[wv][o] = __popcll(m);
      active &= ~m;
    }
    __syncthreads();
    if (valid) {
      int slot = base[own] + rank;
      for (int w = 0; w < wv; ++w) slot += wc[w][own];
      emit(i, slot, own);
    }
    __syncthreads();
    for (int o = threadIdx.x; o < p.W; o += kPT) {
      int sum = 0;
      for (int w = 0; w < kPW; ++w) {
        sum += wc[w][o];
        wc[w][o] = 0;
      }
      base[o] += sum;
    }
    __syncthreads();
  }
}

// ---- document placement (pipeline.common.place_docs) ---------------------------------------------
__device__ __forceinline__ int64_t lower_bound64(const int64_t* __restrict__ a, int64_t n, int64_t x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// hash bucket of a u32 document key: ((key · 0x9E3779B1) mod 2^32 >> 16) mod B (common.doc_owner)
__device__ __forceinline__ int doc_bucket(int64_t key, int B) {
  return (int)((((uint32_t)(uint64_t)key * 0x9E3779B1u) >> 16) % (uint32_t)B);
}

constexpr int kLdsBuckets = 4096;

// both[j] = count of candidate j (0 when absent here), both[nc + b] = Σ counts of the
// non-candidate documents in bucket b. Integer sums: the result does not depend on atomic order.
__global__ __launch_bounds__(256) void k_place_stats(const int64_t* __restrict__ ukeys, const int64_t* __restrict__ ucnt,
                                                     int64_t U, const int64_t* __restrict__ cand, int64_t nc, int B,
                                                     unsigned long long* __restrict__ both) {
  __shared__ unsigned long long hb[kLdsBuckets];
  const bool lds = B <= kLdsBuckets;
  if (lds)
    for (int b = threadIdx.x; b < B; b += 256) hb[b] = 0ull;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x; d < U; d += stride) {
    const int64_t key = ukeys[d];
    const int64_t j = lower_bound64(cand, nc, key);
    const unsigned long long c = (unsigned long long)ucnt[d];
    if (j < nc && cand[j] == key) {
      both[j] = c;
    } else if (c) {
      const int b = doc_bucket(key, B);
      if (lds) atomicAdd(&hb[b], c);
      else atomicAdd(&both[nc + b], c);
    }
  }
  if (lds) {
    __syncthreads();
    for (int b = threadIdx.x; b < B; b += 256)
      if (hb[b]) atomicAdd(&both[nc + b], hb[b]);
  }
}

__global__ __launch_bounds__(256) void k_place_owner(const int64_t* __restrict__ ukeys, int64_t U,
                                                     const int64_t* __restrict__ cand, int64_t nc,
                                                     const int32_t* __restrict__ cown, int B,
                                                     const int32_t* __restrict__ bown, int32_t* __restrict__ uown) {
  const int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (d >= U) return;
  const int64_t key = ukeys[d];
  const int64_t j = lower_bound64(cand, nc, key);
  uown[d] = (j < nc && cand[j] == key) ? cown[j] : bown[doc_bucket(key, B)];
}

#define ONI_TRY(x)                          \
  do {                                       \
    const hipError_t e_ = (x);               \
    if (e_ != hipSuccess) return (int)e_;    \
  } while (0)

}  // namespace

// Stable partition of n items by owner (≤ 256 owners): per-tile histogram, one exclusive scan of
// the owner-major (owner, tile) counts, scatter. counts[W] (int64) gets the items per owner.
template <class Emit>
static int partition_impl(const PartIn& pin, int64_t* counts, void* tmp, size_t* tmp_bytes, hipStream_t s,
                          int32_t** off_out, Emit (*make)(const int32_t* off, void* ctx), void* ctx) {
  const int64_t cells = (int64_t)pin.W * pin.nb;
  Arena ar{static_cast<char*>(tmp)};
  int32_t* blkcnt = ar.take<int32_t>(cells);
  int32_t* off = ar.take<int32_t>(cells);
  size_t sb = 0;
  ONI_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, sb, blkcnt, off, (int)cells, s));
  void* cub = ar.take<char>(sb);
  if (!tmp) {
    *tmp_bytes = ar.used + 256;
    return 0;
  }
  ONI_TRY(hipMemsetAsync(counts, 0, sizeof(int64_t) * pin.W, s));
  if (pin.n == 0) return (int)hipGetLastError();
  k_part_hist<<<pin.nb, kPT, 0, s>>>(pin, blkcnt, reinterpret_cast<unsigned long long*>(counts));
  ONI_TRY(hipcub::DeviceScan::ExclusiveSum(cub, sb, blkcnt, off, (int)cells, s));
  if (off_out) *off_out = off;
  k_part_scatter<<<pin.nb, kPT, 0, s>>>(pin, off, make(off, ctx));
  return (int)hipGetLastError();
}

static bool part_shape_ok(int64_t n, int W) {
  return n >= 0 && n < ((int64_t)1 << 31) && W >= 1 && W <= 256 &&
         (int64_t)W * ((n + kTile - 1) / kTile) < ((int64_t)1 << 31);
}

static PartIn part_in(const int32_t* owner_of_id, const int32_t* ids, int64_t n, int W) {
  return PartIn{owner_of_id, ids, n, W, (int)((n + kTile - 1) / kTile > 0 ? (n + kTile - 1) / kTile : 1)};
}

// owner_of_id[U]: owner rank of each local document id; ids[n]: document id of every token;
// keys[n]: the documents' u32 keys (int64 storage); word[n]; weight[n] or null.
// Outputs: send[n * (weight ? 3 : 2)] grouped by owner rank (stable), order[n] (token of each
// send slot), counts[W] (tokens per owner). W ≤ 256.
// doc_val (optional, int32 [U]): column 0 carries doc_val[ids[t]] instead of the token's key.
struct RouteCtx {
  int32_t* order;
  int32_t* send;
  const int64_t* keys;
  const int32_t* ids;
  const int32_t* doc_val;
  const int32_t* word;
  const int32_t* weight;
};

template <int C, bool DOCVAL>
static EmitRoute<C, DOCVAL> make_route(const int32_t*, void* ctx) {
  const RouteCtx& c = *static_cast<RouteCtx*>(ctx);
  return EmitRoute<C, DOCVAL>{c.order, c.send, c.keys, c.ids, c.doc_val, c.word, c.weight};
}

static int route_pack_impl(const int32_t* owner_of_id, const int32_t* ids, const int64_t* keys,
                           const int32_t* doc_val, const int32_t* word, const int32_t* weight, int64_t n, int W,
                           int32_t* send, int32_t* order, int64_t* counts, void* tmp, size_t* tmp_bytes,
                           hipStream_t s) {
  if (!part_shape_ok(n, W)) return (int)hipErrorInvalidValue;
  const PartIn pin = part_in(owner_of_id, ids, n, W);
  RouteCtx ctx{order, send, keys, ids, doc_val, word, weight};
  if (doc_val) {
    if (weight) return partition_impl(pin, counts, tmp, tmp_bytes, s, nullptr, make_route<3, true>, &ctx);
    return partition_impl(pin, counts, tmp, tmp_bytes, s, nullptr, make_route<2, true>, &ctx);
  }
  if (weight) return partition_impl(pin, counts, tmp, tmp_bytes, s, nullptr, make_route<3, false>, &ctx);
  return partition_impl(pin, counts, tmp, tmp_bytes, s, nullptr, make_route<2, false>, &ctx);
}

ONI_API int oni_route_pack(const int32_t* owner_of_id, const int32_t* ids, const int64_t* keys, const int32_t* word,
                           const int32_t* weight, int64_t n, int W, int32_t* send, int32_t* order, int64_t* counts,
                           void* tmp, size_t* tmp_bytes, hipStream_t s) {
  return route_pack_impl(owner_of_id, ids, keys, nullptr, word, weight, n, W, send, order, counts, tmp, tmp_bytes, s);
}

ONI_API int oni_route_pack_ids(const int32_t* owner_of_id, const int32_t* ids, const int32_t* doc_val,
                               const int32_t* word, const int32_t* weight, int64_t n, int W, int32_t* send,
                               int32_t* order, int64_t* counts, void* tmp, size_t* tmp_bytes, hipStream_t s) {
  return route_pack_impl(owner_of_id, ids, nullptr, doc_val, word, weight, n, W, send, order, counts, tmp, tmp_bytes,
                         s);
}

// recv[n * C] rows grouped by source rank (seg[W + 1] row offsets), column 0 an index into that
// source's key list; kid: dictionary id of every entry of the concatenated key lists, koff[W]: the
// start of each source's list in it. Outputs doc/word (and wt, optional) int32 [n].
ONI_API int oni_route_unpack(const int32_t* recv, int64_t n, int C, const int64_t* seg, const int64_t* koff, int W,
                             const int32_t* kid, int32_t* doc, int32_t* word, int32_t* wt, hipStream_t s) {
  if (W < 1 || W > 256 || (C != 2 && C != 3) || n < 0) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  k_route_unpack<<<nblk(n), kB, 0, s>>>(recv, n, C, seg, koff, W, kid, doc, word, wt);
  return (int)hipGetLastError();
}

// Stable partition of n items (item i's owner: owner_of_id[ids ? ids[i] : i]) into owner groups:
// order[n] (slot → item), counts[W] (int64), and optionally rank[n] (item → slot within its
// group) and keys_out[n] (u32 bits of keys[i] at its slot). W ≤ 256.
struct PartCtx {
  int32_t* order;
  int32_t* rank;
  const int64_t* keys;
  int32_t* keys_out;
  int nb;
};

static EmitPart make_part(const int32_t* off, void* ctx) {
  const PartCtx& c = *static_cast<PartCtx*>(ctx);
  return EmitPart{c.order, c.rank, c.keys, c.keys_out, off, c.nb};
}

ONI_API int oni_partition(const int32_t* owner_of_id, const int32_t* ids, const int64_t* keys, int64_t n, int W,
                          int32_t* order, int32_t* rank, int32_t* keys_out, int64_t* counts, void* tmp,
                          size_t* tmp_bytes, hipStream_t s) {
  if (!part_shape_ok(n, W) || (keys_out && !keys && n > 0)) return (int)hipErrorInvalidValue;
  const PartIn pin = part_in(owner_of_id, ids, n, W);
  PartCtx ctx{order, rank, keys, keys_out, pin.nb};
  return partition_impl(pin, counts, tmp, tmp_bytes, s, nullptr, make_part, &ctx);
}

// place_docs bookkeeping. ukeys[U] ascending, ucnt[U]; cand[nc] ascending. both[nc + B] (int64) is
// overwritten: candidate counts, then the bucket loads of the other documents.
ONI_API int oni_place_stats(const int64_t* ukeys, const int64_t* ucnt, int64_t U, const int64_t* cand, int64_t nc,
                            int B, int64_t* both, hipStream_t s) {
  if (U < 0 || nc < 0 || B < 1) return (int)hipErrorInvalidValue;
  ONI_TRY(hipMemsetAsync(both, 0, sizeof(int64_t) * (size_t)(nc + B), s));
  if (U == 0) return (int)hipGetLastError();
  const unsigned g = oni::grid_for(U, 256, 1024);
  k_place_stats<<<g, 256, 0, s>>>(ukeys, ucnt, U, cand, nc, B, reinterpret_cast<unsigned long long*>(both));
  return (int)hipGetLastError();
}

// uown[d] = cown[j] when ukeys[d] == cand[j], else bown[bucket of ukeys[d]].
ONI_API int oni_place_owner(const int64_t* ukeys, int64_t U, const int64_t* cand, int64_t nc, const int32_t* cown,
                            int B, const int32_t* bown, int32_t* uown, hipStream_t s) {
  if (U < 0 || nc < 0 || B < 1) return (int)hipErrorInvalidValue;
  if (U == 0) return 0;
  k_place_owner<<<nblk(U), 256, 0, s>>>(ukeys, U, cand, nc, cown, B, bown, uown);
  return (int)hipGetLastError();
}
