// K08 / K09 -- dictionary encoding and the document-term corpus build, on device.
//
// Replaces oni-ml's `zipWithIndex` dictionaries and `reduceByKey((ip, word) -> count)` + lda-c
// `model.dat` writer (OniLDACWrapper.createModel, SURVEY.md §2.2 C20, [U-M]): instead of a Spark
// shuffle, every stage is a radix sort (rocPRIM onesweep through hipCUB, sorting only the key bits
// that can be non-zero) followed by flag-heads → scan → scatter kernels. The host reads back three
// small scalars in total (dictionary sizes, pair count + token/chunk totals, SELL size); every
// other size is consumed on the device.
//
//   dict_encode   u64 keys → sorted unique keys + dense id of every key (inverse map)
//   pair_build    (doc id, word id[, weight]) tokens → sorted distinct (doc, word) pairs, their
//                 counts (Σ weights: feedback duplication is a count bump, C19), the pair index of
//                 every token (the score plan's event → pair map, K15) and the side-0 event order
//   doc_layout    CSR: doc_pair_ptr, doc_tok_ptr, pair_tokoff; chunks per doc (≤ L tokens each)
//   chunk_layout  chunks sorted longest first (stable) and packed S to a SELL slice
//   word_index    word-sorted token index of the SELL layout (wsorted, wslot, wpos, recount tiles)
//
// Every launcher takes a scratch buffer; called with tmp == nullptr it only reports the bytes it
// needs. Bitwise contract: the outputs equal the torch reference build (oni355/models/corpus.py
// build_corpus) field by field (tests/test_gpu_kernels.py).
#include <hipcub/hipcub.hpp>

#include "oni_common.h"

namespace {

constexpr int kB = 256;
inline unsigned nblk(int64_t n) { return (unsigned)((n + kB - 1) / kB > 0 ? (n + kB - 1) / kB : 1); }

// bump allocator over the caller's scratch buffer (256-B aligned slices)
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

__global__ void k_iota(int32_t* __restrict__ v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) v[i] = (int32_t)i;
}

template <class K>
__global__ void k_heads(const K* __restrict__ k, int64_t n, int32_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) flag[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

// keys of at most 32 significant bits are sorted as u32: a radix pass then moves 8 B per element
// (key + index) instead of 12
__global__ void k_narrow(const uint64_t* __restrict__ k, int64_t n, uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) out[i] = (uint32_t)k[i];
}

// The id of every key in input order is the inverse permutation applied to the sorted ranks. As
// one scatter (ids[perm[i]] = r) every 4-B store lands on its own line: 25M of them cost ~0.55 ms.
// Above kSortBackMin keys the ranks are written in sorted order (SEQ), ONE radix pass over perm's
// top 8 bits groups them into 256 destination windows (~0.4 MB each at 25M), and the scatter then
// writes inside a window at a time, where the L2 merges the stores into whole lines.
constexpr int64_t kSortBackMin = int64_t(1) << 21;

template <class K, bool SEQ>
__global__ void k_dict_scatter(const K* __restrict__ ks, const int32_t* __restrict__ perm,
                               const int32_t* __restrict__ rank, int64_t n, uint64_t* __restrict__ uniq,
                               int32_t* __restrict__ ids, int64_t* __restrict__ n_uniq, int64_t* __restrict__ head) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  const int32_t r = rank[i] - 1;
  if constexpr (SEQ) ids[i] = r;
  else ids[perm[i]] = r;
  if (i == 0 || ks[i] != ks[i - 1]) {
    uniq[r] = (uint64_t)ks[i];
    if (head) head[r] = i;
  }
  if (i == n - 1) {
    *n_uniq = (int64_t)r + 1;
    if (head) head[r + 1] = n;
  }
}

template <class K>
__global__ void k_pair_keys(const int32_t* __restrict__ doc, const int32_t* __restrict__ word, int64_t n, int64_t V,
                            K* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) key[i] = (K)((uint64_t)doc[i] * (uint64_t)V + (uint64_t)word[i]);
}

template <class K, bool SEQ>
__global__ void k_pair_scatter(const K* __restrict__ ks, const int32_t* __restrict__ perm,
                               const int32_t* __restrict__ run, int64_t n, int64_t V, int32_t* __restrict__ pair_doc,
                               int32_t* __restrict__ pair_word, int64_t* __restrict__ head_pos,
                               int32_t* __restrict__ tok_pair, int64_t* __restrict__ nnz) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  const int32_t r = run[i] - 1;
  if constexpr (SEQ) tok_pair[i] = r;  // sorted order: scatter_back restores the token order
  else tok_pair[perm[i]] = r;
  if (i == 0 || ks[i] != ks[i - 1]) {
    pair_doc[r] = (int32_t)((uint64_t)ks[i] / (uint64_t)V);
    pair_word[r] = (int32_t)((uint64_t)ks[i] % (uint64_t)V);
    head_pos[r] = i;
  }
  if (i == n - 1) {
    *nnz = (int64_t)r + 1;
    head_pos[r + 1] = n;
  }
}

__global__ void k_weights_sorted(const int32_t* __restrict__ w, const int32_t* __restrict__ perm, int64_t n,
                                 int64_t* __restrict__ ws) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) ws[i] = w ? (int64_t)w[perm[i]] : 1;
}

// cnt[r] = Σ weights of run r (psum = inclusive prefix of the sorted weights)
__global__ void k_pair_counts(const int64_t* __restrict__ head_pos, const int64_t* __restrict__ psum,
                              const int64_t* __restrict__ nnz_p, int64_t n, int32_t* __restrict__ cnt) {
  const int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (r >= *nnz_p) return;
  const int64_t a = head_pos[r], b = head_pos[r + 1];
  const int64_t s = psum ? psum[b - 1] - (a > 0 ? psum[a - 1] : 0) : b - a;  // no weights: run length
  cnt[r] = (int32_t)(s < 0x7FFFFFFF ? s : 0x7FFFFFFF);
}

// sums[r] = Σ sorted weights of run r (64-bit; dictionary counts)
__global__ void k_run_sums(const int64_t* __restrict__ head_pos, const int64_t* __restrict__ psum,
                           const int64_t* __restrict__ nr_p, int64_t* __restrict__ sums) {
  const int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (r >= *nr_p) return;
  const int64_t a = head_pos[r], b = head_pos[r + 1];
  sums[r] = psum ? psum[b - 1] - (a > 0 ? psum[a - 1] : 0) : b - a;  // no weights: run length
}

struct BelowN {
  int32_t n0;
  __host__ __device__ bool operator()(const int32_t& v) const { return v < n0; }
};

// doc_pair_ptr[d] = first pair of doc d (pairs are doc-major; empty docs point at the next one)
__global__ void k_doc_pair_ptr(const int32_t* __restrict__ pair_doc, int64_t nnz, int64_t D,
                               int64_t* __restrict__ ptr) {
  const int64_t j = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (j >= nnz) return;
  const int64_t d = pair_doc[j];
  const int64_t prev = j == 0 ? -1 : pair_doc[j - 1];
  for (int64_t e = prev + 1; e <= d; ++e) ptr[e] = j;
  if (j == nnz - 1)
    for (int64_t e = d + 1; e <= D; ++e) ptr[e] = nnz;
}

__global__ void k_i32_to_i64(const int32_t* __restrict__ a, int64_t n, int64_t* __restrict__ b) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) b[i] = a[i];
  if (i == n) b[i] = 0;
}

// doc_tok_ptr[d] = glob[doc_pair_ptr[d]]; per-doc token count and chunk count
__global__ void k_doc_tok(const int64_t* __restrict__ pair_ptr, const int64_t* __restrict__ glob, int64_t D, int L,
                          int64_t* __restrict__ tok_ptr, int64_t* __restrict__ nch, int32_t* __restrict__ is_long) {
  const int64_t d = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (d > D) return;
  tok_ptr[d] = glob[pair_ptr[d]];
  if (d == D) {
    nch[D] = 0;
    return;
  }
  const int64_t nt = glob[pair_ptr[d + 1]] - glob[pair_ptr[d]];
  const int64_t c = (nt + L - 1) / L;
  nch[d] = c;
  is_long[d] = c > 1 ? 1 : 0;
}

__global__ void k_pair_tokoff(const int32_t* __restrict__ pair_doc, const int64_t* __restrict__ glob,
                              const int64_t* __restrict__ tok_ptr, int64_t nnz, int64_t* __restrict__ tokoff) {
  const int64_t j = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (j < nnz) tokoff[j] = glob[j] - tok_ptr[pair_doc[j]];
}

__global__ void k_scalars3(const int64_t* __restrict__ a, const int64_t* __restrict__ b, const int32_t* __restrict__ c,
                           int64_t* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = *a;
    out[1] = *b;
    out[2] = (int64_t)*c;
  }
}

// one thread per chunk: doc = upper_bound(chunk_first, i) - 1
__global__ void k_chunks(const int64_t* __restrict__ chunk_first, const int64_t* __restrict__ tok_ptr, int64_t D,
                         int64_t n_chunks, int L, int32_t* __restrict__ cdoc, int32_t* __restrict__ cpos0,
                         int32_t* __restrict__ clen, uint8_t* __restrict__ cmulti, uint32_t* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i >= n_chunks) return;
  int64_t lo = 0, hi = D;  // invariant: chunk_first[lo] <= i < chunk_first[hi]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (chunk_first[mid] <= i) lo = mid; else hi = mid;
  }
  const int64_t c = i - chunk_first[lo];
  const int64_t nt = tok_ptr[lo + 1] - tok_ptr[lo];
  const int64_t p0 = c * L;
  const int64_t ln = nt - p0 < L ? nt - p0 : L;
  cdoc[i] = (int32_t)lo;
  cpos0[i] = (int32_t)p0;
  clen[i] = (int32_t)ln;
  cmulti[i] = (chunk_first[lo + 1] - chunk_first[lo]) > 1 ? 1 : 0;
  key[i] = (uint32_t)(L - ln);
}

// gather the length-sorted chunks into the padded [ns*S] tables (pads: doc -1, len 0)
__global__ void k_chunk_gather(const int32_t* __restrict__ order, int64_t n_chunks, int64_t n_pad_total,
                               const int32_t* __restrict__ cdoc, const int32_t* __restrict__ cpos0,
                               const int32_t* __restrict__ clen, const uint8_t* __restrict__ cmulti,
                               const int32_t* __restrict__ doc_keys, int32_t* __restrict__ o_doc,
                               int32_t* __restrict__ o_pos0, int32_t* __restrict__ o_len, uint8_t* __restrict__ o_multi,
                               int32_t* __restrict__ o_key) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i >= n_pad_total) return;
  if (i < n_chunks) {
    const int32_t s = order[i];
    const int32_t d = cdoc[s];
    o_doc[i] = d;
    o_pos0[i] = cpos0[s];
    o_len[i] = clen[s];
    o_multi[i] = cmulti[s];
    o_key[i] = doc_keys[d];
  } else {
    o_doc[i] = -1;
    o_pos0[i] = 0;
    o_len[i] = 0;
    o_multi[i] = 0;
    o_key[i] = 0;
  }
}

__global__ void k_slice_len(const int32_t* __restrict__ o_len, int64_t ns, int S, int32_t* __restrict__ slice_len,
                            int64_t* __restrict__ slice_w) {
  const int64_t s = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (s < ns) {
    slice_len[s] = o_len[s * S];
    slice_w[s] = (int64_t)o_len[s * S] * S;
  }
  if (s == ns) slice_w[ns] = 0;
}

__global__ void k_word_keys(const uint32_t* __restrict__ tok_word, int64_t n, uint32_t V, uint32_t* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) {
    const uint32_t w = tok_word[i];
    key[i] = w == oni::kPadWord ? V : w;
  }
}

// the sort wrote wsorted / wslot in place (their first T entries are the real tokens, padding
// sorts last under key V): what is left is the inverse map and the recount tile bounds
__global__ void k_word_index(const uint32_t* __restrict__ ks, const int32_t* __restrict__ slot, int64_t T, int tile,
                             int32_t* __restrict__ wpos, int32_t* __restrict__ tile_wlo,
                             int32_t* __restrict__ tile_whi) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i >= T) return;
  wpos[slot[i]] = (int32_t)i;
  if (i % tile == 0) {
    const int64_t t = i / tile;
    const int64_t e = i + tile - 1 < T - 1 ? i + tile - 1 : T - 1;
    tile_wlo[t] = (int32_t)ks[i];
    tile_whi[t] = (int32_t)ks[e];
  }
}

__global__ void k_fill_i32(int32_t* __restrict__ p, int64_t n, int32_t v) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) p[i] = v;
}

#define ONI_TRY(x)                          \
  do {                                       \
    const hipError_t e_ = (x);               \
    if (e_ != hipSuccess) return (int)e_;    \
  } while (0)

int bits_for(uint64_t maxv) {  // number of bits needed to represent values in [0, maxv]
  int b = 1;
  while (b < 64 && (maxv >> b)) ++b;
  return b;
}

// one radix pass of (perm, val) over perm's top 8 bits: destination windows of 2^(bits-8) slots
hipError_t window_pass(void* tmp, size_t& bytes, const int32_t* perm, int32_t* keys_out, const int32_t* val,
                       int32_t* val_out, int64_t n, hipStream_t s) {
  const int pbits = bits_for(n > 1 ? (uint64_t)(n - 1) : 1);
  const int lo = pbits > 8 ? pbits - 8 : 0;
  return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, reinterpret_cast<const uint32_t*>(perm),
                                            reinterpret_cast<uint32_t*>(keys_out), val, val_out, (int)n, lo, pbits,
                                            s);
}

// XCD-aware: workgroups are dispatched round-robin over the 8 XCDs, so workgroup b takes tile
// (b % 8) * (grid / 8) + b / 8 -- each XCD walks one contiguous eighth of the window-grouped
// input, and a destination window's lines fill in ONE L2 instead of eight partial copies.
__global__ void k_scatter(const int32_t* __restrict__ dst, const int32_t* __restrict__ val, int64_t n,
                          int32_t* __restrict__ out) {
  const unsigned per = gridDim.x / 8u;  // grid is a multiple of 8
  const unsigned t = (blockIdx.x % 8u) * per + blockIdx.x / 8u;
  const int64_t i = (int64_t)t * kB + threadIdx.x;
  if (i < n) out[dst[i]] = val[i];
}

inline unsigned nblk8(int64_t n) { return (nblk(n) + 7u) & ~7u; }

}  // namespace

// ------------------------------------------------------------------------------------------------
// dict_encode: keys[n] (u64) → uniq (sorted, n_uniq on device) + ids[n] (int32 rank of each key)
// Optional counts[n] (int64): Σ weight (1 per key without ``weight``) of every unique key -- the
// per-document token counts the data-parallel placement needs, read off the sorted runs instead of
// a same-address-atomic index_add (power-law documents serialise those: 12 ms at 25M tokens).
template <class K>
static int dict_encode_impl(const uint64_t* keys, int64_t n, int key_bits, uint64_t* uniq, int32_t* ids,
                            int64_t* n_uniq, const int32_t* weight, int64_t* counts, void* tmp, size_t* tmp_bytes,
                            hipStream_t s) {
  constexpr bool kNarrow = sizeof(K) == 4;
  Arena ar{static_cast<char*>(tmp)};
  K* kin = kNarrow ? ar.take<K>(n) : nullptr;
  K* ks = ar.take<K>(n);
  int32_t* iota = ar.take<int32_t>(n);
  int32_t* perm = ar.take<int32_t>(n);
  int32_t* flag = ar.take<int32_t>(n);
  int32_t* rank = ar.take<int32_t>(n);
  int64_t* head = counts ? ar.take<int64_t>(n + 1) : nullptr;
  int64_t* ws = counts ? ar.take<int64_t>(n) : nullptr;
  int64_t* psum = counts ? ar.take<int64_t>(n) : nullptr;
  const K* src = kNarrow ? kin : reinterpret_cast<const K*>(keys);
  size_t sb = 0, cb = 0, wb = 0, bb = 0;
  const bool back = n >= kSortBackMin;
  // window pass scratch: keys into iota (free after the sort), values into a slice of its own
  int32_t* wval = back ? ar.take<int32_t>(n) : nullptr;
  ONI_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, sb, src, ks, iota, perm, (int)n, 0, key_bits, s));
  ONI_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, cb, flag, rank, (int)n, s));
  if (counts) ONI_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, wb, ws, psum, (int)n, s));
  if (back) ONI_TRY(window_pass(nullptr, bb, perm, iota, flag, wval, n, s));
  size_t cbytes = sb > cb ? sb : cb;
  if (wb > cbytes) cbytes = wb;
  if (bb > cbytes) cbytes = bb;
  void* cub = ar.take<char>(cbytes);
  if (!tmp) {
    *tmp_bytes = ar.used + 256;
    return 0;
  }
  if (n == 0) {
    ONI_TRY(hipMemsetAsync(n_uniq, 0, sizeof(int64_t), s));
    return (int)hipGetLastError();
  }
  if constexpr (kNarrow) k_narrow<<<nblk(n), kB, 0, s>>>(keys, n, reinterpret_cast<uint32_t*>(kin));
  k_iota<<<nblk(n), kB, 0, s>>>(iota, n);
  ONI_TRY(hipcub::DeviceRadixSort::SortPairs(cub, cbytes, src, ks, iota, perm, (int)n, 0, key_bits, s));
  k_heads<K><<<nblk(n), kB, 0, s>>>(ks, n, flag);
  ONI_TRY(hipcub::DeviceScan::InclusiveSum(cub, cbytes, flag, rank, (int)n, s));
  if (back) {
    // ranks in sorted order into flag (free after the scan), grouped by destination window, placed
    k_dict_scatter<K, true><<<nblk(n), kB, 0, s>>>(ks, perm, rank, n, uniq, flag, n_uniq, head);
    ONI_TRY(window_pass(cub, cbytes, perm, iota, flag, wval, n, s));
    k_scatter<<<nblk8(n), kB, 0, s>>>(iota, wval, n, ids);
  } else {
    k_dict_scatter<K, false><<<nblk(n), kB, 0, s>>>(ks, perm, rank, n, uniq, ids, n_uniq, head);
  }
  if (counts) {
    // unweighted keys count their run lengths: no 8-B-per-key weight stream and scan
    if (weight) {
      k_weights_sorted<<<nblk(n), kB, 0, s>>>(weight, perm, n, ws);
      ONI_TRY(hipcub::DeviceScan::InclusiveSum(cub, cbytes, ws, psum, (int)n, s));
    }
    k_run_sums<<<nblk(n), kB, 0, s>>>(head, weight ? psum : nullptr, n_uniq, counts);
  }
  return (int)hipGetLastError();
}

ONI_API int oni_dict_encode(const uint64_t* keys, int64_t n, int key_bits, uint64_t* uniq, int32_t* ids,
                            int64_t* n_uniq, const int32_t* weight, int64_t* counts, void* tmp, size_t* tmp_bytes,
                            hipStream_t s) {
  if (n >= (int64_t)1 << 31) return (int)hipErrorInvalidValue;
  if (key_bits <= 32)
    return dict_encode_impl<uint32_t>(keys, n, key_bits, uniq, ids, n_uniq, weight, counts, tmp, tmp_bytes, s);
  return dict_encode_impl<uint64_t>(keys, n, key_bits, uniq, ids, n_uniq, weight, counts, tmp, tmp_bytes, s);
}

// ------------------------------------------------------------------------------------------------
// pair_build: tokens (doc, word[, weight]) → distinct pairs (doc-major, word-sorted) with counts,
// tok_pair[n] (pair of every token), nnz on device; order0[n0] = tokens < n0 sorted by pair
// (stable: the score plan's first-endpoint event order). Outputs sized n (nnz ≤ n).
template <class K>
static int pair_build_impl(const int32_t* doc, const int32_t* word, const int32_t* weight, int64_t n, int64_t V,
                           int bits, int32_t* pair_doc, int32_t* pair_word, int32_t* pair_cnt, int32_t* tok_pair,
                           int64_t* nnz, int32_t* order0, int64_t n0, void* tmp, size_t* tmp_bytes, hipStream_t s) {
  Arena ar{static_cast<char*>(tmp)};
  K* key = ar.take<K>(n);
  K* ks = ar.take<K>(n);
  int32_t* iota = ar.take<int32_t>(n);
  int32_t* perm = ar.take<int32_t>(n);
  int32_t* flag = ar.take<int32_t>(n);
  int32_t* run = ar.take<int32_t>(n);
  int64_t* head = ar.take<int64_t>(n + 1);
  int64_t* ws = ar.take<int64_t>(n);
  int64_t* psum = ar.take<int64_t>(n);
  int64_t* nsel = ar.take<int64_t>(1);
  size_t b1 = 0, b2 = 0, b3 = 0, b4 = 0, b5 = 0;
  const bool back = n >= kSortBackMin;
  int32_t* wval = back ? ar.take<int32_t>(n) : nullptr;
  if (back) ONI_TRY(window_pass(nullptr, b5, perm, iota, flag, wval, n, s));
  ONI_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, key, ks, iota, perm, (int)n, 0, bits, s));
  ONI_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, b2, flag, run, (int)n, s));
  ONI_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, b3, ws, psum, (int)n, s));
  ONI_TRY(hipcub::DeviceSelect::If(nullptr, b4, perm, order0, nsel, (int)n, BelowN{(int32_t)n0}, s));
  size_t cbytes = b1;
  if (b2 > cbytes) cbytes = b2;
  if (b3 > cbytes) cbytes = b3;
  if (b4 > cbytes) cbytes = b4;
  if (b5 > cbytes) cbytes = b5;
  void* cub = ar.take<char>(cbytes);
  if (!tmp) {
    *tmp_bytes = ar.used + 256;
    return 0;
  }
  if (n == 0) {
    ONI_TRY(hipMemsetAsync(nnz, 0, sizeof(int64_t), s));
    return (int)hipGetLastError();
  }
  k_pair_keys<K><<<nblk(n), kB, 0, s>>>(doc, word, n, V, key);
  k_iota<<<nblk(n), kB, 0, s>>>(iota, n);
  ONI_TRY(hipcub::DeviceRadixSort::SortPairs(cub, cbytes, key, ks, iota, perm, (int)n, 0, bits, s));
  k_heads<K><<<nblk(n), kB, 0, s>>>(ks, n, flag);
  ONI_TRY(hipcub::DeviceScan::InclusiveSum(cub, cbytes, flag, run, (int)n, s));
  if (back) {
    k_pair_scatter<K, true><<<nblk(n), kB, 0, s>>>(ks, perm, run, n, V, pair_doc, pair_word, head, flag, nnz);
    ONI_TRY(window_pass(cub, cbytes, perm, iota, flag, wval, n, s));
    k_scatter<<<nblk8(n), kB, 0, s>>>(iota, wval, n, tok_pair);
  } else {
    k_pair_scatter<K, false><<<nblk(n), kB, 0, s>>>(ks, perm, run, n, V, pair_doc, pair_word, head, tok_pair, nnz);
  }
  if (weight) {
    k_weights_sorted<<<nblk(n), kB, 0, s>>>(weight, perm, n, ws);
    ONI_TRY(hipcub::DeviceScan::InclusiveSum(cub, cbytes, ws, psum, (int)n, s));
  }
  k_pair_counts<<<nblk(n), kB, 0, s>>>(head, weight ? psum : nullptr, nnz, n, pair_cnt);
  if (order0 && n0 > 0) ONI_TRY(hipcub::DeviceSelect::If(cub, cbytes, perm, order0, nsel, (int)n, BelowN{(int32_t)n0}, s));
  return (int)hipGetLastError();
}

ONI_API int oni_pair_build(const int32_t* doc, const int32_t* word, const int32_t* weight, int64_t n, int64_t D,
                           int64_t V, int32_t* pair_doc, int32_t* pair_word, int32_t* pair_cnt, int32_t* tok_pair,
                           int64_t* nnz, int32_t* order0, int64_t n0, void* tmp, size_t* tmp_bytes, hipStream_t s) {
  if (n >= (int64_t)1 << 31) return (int)hipErrorInvalidValue;
  const int bits = bits_for((uint64_t)(D > 0 ? D : 1) * (uint64_t)(V > 0 ? V : 1));
  if (bits <= 32)
    return pair_build_impl<uint32_t>(doc, word, weight, n, V, bits, pair_doc, pair_word, pair_cnt, tok_pair, nnz,
                                     order0, n0, tmp, tmp_bytes, s);
  return pair_build_impl<uint64_t>(doc, word, weight, n, V, bits, pair_doc, pair_word, pair_cnt, tok_pair, nnz,
                                   order0, n0, tmp, tmp_bytes, s);
}

// ------------------------------------------------------------------------------------------------
// doc_layout: CSR pointers + chunk counts. scalars[3] ← (T, n_chunks, n_long_docs).
// Outputs: doc_pair_ptr[D+1], doc_tok_ptr[D+1], pair_tokoff[nnz], chunk_first[D+1], long_rows[D]
ONI_API int oni_doc_layout(const int32_t* pair_doc, const int32_t* pair_cnt, int64_t nnz, int64_t D, int L,
                           int64_t* doc_pair_ptr, int64_t* doc_tok_ptr, int64_t* pair_tokoff, int64_t* chunk_first,
                           int32_t* long_rows, int64_t* scalars, void* tmp, size_t* tmp_bytes, hipStream_t s) {
  Arena ar{static_cast<char*>(tmp)};
  int64_t* c64 = ar.take<int64_t>(nnz + 1);
  int64_t* glob = ar.take<int64_t>(nnz + 1);
  int64_t* nch = ar.take<int64_t>(D + 1);
  int32_t* is_long = ar.take<int32_t>(D + 1);
  int32_t* iota = ar.take<int32_t>(D + 1);
  int32_t* n_long = ar.take<int32_t>(1);
  size_t b1 = 0, b2 = 0, b3 = 0;
  ONI_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, b1, c64, glob, (int)(nnz + 1), s));
  ONI_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, b2, nch, chunk_first, (int)(D + 1), s));
  ONI_TRY(hipcub::DeviceSelect::Flagged(nullptr, b3, iota, is_long, long_rows, n_long, (int)D, s));
  size_t cbytes = b1 > b2 ? b1 : b2;
  if (b3 > cbytes) cbytes = b3;
  void* cub = ar.take<char>(cbytes);
  if (!tmp) {
    *tmp_bytes = ar.used + 256;
    return 0;
  }
  if (nnz > 0) k_doc_pair_ptr<<<nblk(nnz), kB, 0, s>>>(pair_doc, nnz, D, doc_pair_ptr);
  else k_fill_i32<<<1, kB, 0, s>>>(reinterpret_cast<int32_t*>(doc_pair_ptr), 2 * (D + 1), 0);
  k_i32_to_i64<<<nblk(nnz + 1), kB, 0, s>>>(pair_cnt, nnz, c64);
  ONI_TRY(hipcub::DeviceScan::ExclusiveSum(cub, cbytes, c64, glob, (int)(nnz + 1), s));
  k_doc_tok<<<nblk(D + 1), kB, 0, s>>>(doc_pair_ptr, glob, D, L, doc_tok_ptr, nch, is_long);
  k_pair_tokoff<<<nblk(nnz), kB, 0, s>>>(pair_doc, glob, doc_tok_ptr, nnz, pair_tokoff);
  ONI_TRY(hipcub::DeviceScan::ExclusiveSum(cub, cbytes, nch, chunk_first, (int)(D + 1), s));
  k_iota<<<nblk(D), kB, 0, s>>>(iota, D);
  if (D > 0) ONI_TRY(hipcub::DeviceSelect::Flagged(cub, cbytes, iota, is_long, long_rows, n_long, (int)D, s));
  else ONI_TRY(hipMemsetAsync(n_long, 0, sizeof(int32_t), s));
  k_scalars3<<<1, 64, 0, s>>>(glob + nnz, chunk_first + D, n_long, scalars);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// chunk_layout: chunks (≤ L tokens of one doc) sorted by length, longest first (stable), padded
// to ns*S. Outputs [ns*S]: chunk_doc, chunk_pos0, chunk_len, chunk_multi, chunk_key; slice_len[ns];
// slice_off[ns+1] (exclusive prefix of slice_len*S: slice_off[ns] = SELL slots).
ONI_API int oni_chunk_layout(const int64_t* chunk_first, const int64_t* doc_tok_ptr, const int32_t* doc_keys,
                             int64_t D, int64_t n_chunks, int L, int S, int32_t* chunk_doc, int32_t* chunk_pos0,
                             int32_t* chunk_len, uint8_t* chunk_multi, int32_t* chunk_key, int32_t* slice_len,
                             int64_t* slice_off, void* tmp, size_t* tmp_bytes, hipStream_t s) {
  const int64_t ns = (n_chunks + S - 1) / S;
  Arena ar{static_cast<char*>(tmp)};
  int32_t* cdoc = ar.take<int32_t>(n_chunks);
  int32_t* cpos0 = ar.take<int32_t>(n_chunks);
  int32_t* clen = ar.take<int32_t>(n_chunks);
  uint8_t* cmul = ar.take<uint8_t>(n_chunks);
  uint32_t* key = ar.take<uint32_t>(n_chunks);
  uint32_t* ks = ar.take<uint32_t>(n_chunks);
  int32_t* iota = ar.take<int32_t>(n_chunks);
  int32_t* order = ar.take<int32_t>(n_chunks);
  int64_t* sw = ar.take<int64_t>(ns + 1);
  const int kbits = bits_for((uint64_t)L);
  size_t b1 = 0, b2 = 0;
  ONI_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, key, ks, iota, order, (int)n_chunks, 0, kbits, s));
  ONI_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, b2, sw, slice_off, (int)(ns + 1), s));
  void* cub = ar.take<char>(b1 > b2 ? b1 : b2);
  if (!tmp) {
    *tmp_bytes = ar.used + 256;
    return 0;
  }
  size_t cbytes = b1 > b2 ? b1 : b2;
  if (n_chunks > 0) {
    k_chunks<<<nblk(n_chunks), kB, 0, s>>>(chunk_first, doc_tok_ptr, D, n_chunks, L, cdoc, cpos0, clen, cmul, key);
    k_iota<<<nblk(n_chunks), kB, 0, s>>>(iota, n_chunks);
    ONI_TRY(hipcub::DeviceRadixSort::SortPairs(cub, cbytes, key, ks, iota, order, (int)n_chunks, 0, kbits, s));
  }
  k_chunk_gather<<<nblk(ns * S), kB, 0, s>>>(order, n_chunks, ns * S, cdoc, cpos0, clen, cmul, doc_keys, chunk_doc,
                                            chunk_pos0, chunk_len, chunk_multi, chunk_key);
  k_slice_len<<<nblk(ns + 1), kB, 0, s>>>(chunk_len, ns, S, slice_len, sw);
  ONI_TRY(hipcub::DeviceScan::ExclusiveSum(cub, cbytes, sw, slice_off, (int)(ns + 1), s));
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// word_index: word-sorted view of the SELL tokens (stable by slot): wsorted, wslot (sized
// ``slots``: the first T entries are the tokens, the sort writes them in place), wpos[slots] (-1 on
// padding), tile_wlo/tile_whi[ceil(T/tile)] (K11 recount tiles)
ONI_API int oni_word_index(const uint32_t* tok_word, int64_t slots, int64_t T, int64_t V, int tile,
                           int32_t* wsorted, int32_t* wslot, int32_t* wpos, int32_t* tile_wlo, int32_t* tile_whi,
                           void* tmp, size_t* tmp_bytes, hipStream_t s) {
  if (slots >= (int64_t)1 << 31) return (int)hipErrorInvalidValue;
  Arena ar{static_cast<char*>(tmp)};
  uint32_t* key = ar.take<uint32_t>(slots);
  uint32_t* ks = reinterpret_cast<uint32_t*>(wsorted);
  int32_t* iota = ar.take<int32_t>(slots);
  int32_t* slot = wslot;
  const int kbits = bits_for((uint64_t)V);
  size_t b1 = 0;
  ONI_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, key, ks, iota, slot, (int)slots, 0, kbits, s));
  void* cub = ar.take<char>(b1);
  if (!tmp) {
    *tmp_bytes = ar.used + 256;
    return 0;
  }
  k_fill_i32<<<nblk(slots), kB, 0, s>>>(wpos, slots, -1);
  if (slots == 0) return (int)hipGetLastError();
  k_word_keys<<<nblk(slots), kB, 0, s>>>(tok_word, slots, (uint32_t)V, key);
  k_iota<<<nblk(slots), kB, 0, s>>>(iota, slots);
  ONI_TRY(hipcub::DeviceRadixSort::SortPairs(cub, b1, key, ks, iota, slot, (int)slots, 0, kbits, s));
  if (T > 0) k_word_index<<<nblk(T), kB, 0, s>>>(ks, slot, T, tile, wpos, tile_wlo, tile_whi);
  return (int)hipGetLastError();
}
