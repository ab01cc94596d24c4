// Data-parallel token routing: pack every token for its document's owner rank.
//
// The reference shipped whole corpus files to the MPI ranks of oni-lda-c ([U-H]). Here each rank
// featurizes its own events and every token (doc key, word id[, weight]) must reach the rank that
// owns its document before the corpus build. route_pack turns "owner of every local document" into
// the all-to-all send buffer in one stable partition: the owner (≤ 8 bits) is the whole radix key,
// so it is a single onesweep pass, followed by one gather that writes the packed int32 columns
// (8 B per token, 12 B with weights, instead of three int64 columns) and an LDS-privatised owner
// histogram for the send counts. ``order`` (slot → token) is what the way back
// (oni355.pipeline.common.return_to_origin) scatters through.
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

__global__ void k_owner_keys(const int32_t* __restrict__ owner_of_id, const int32_t* __restrict__ ids, int64_t n,
                             uint8_t* __restrict__ okey, int32_t* __restrict__ iota) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  okey[i] = (uint8_t)owner_of_id[ids[i]];
  iota[i] = (int32_t)i;
}

// per-block owner histogram in LDS, one global atomic per (block, owner)
__global__ void k_owner_hist(const uint8_t* __restrict__ okey, int64_t n, int W,
                             unsigned long long* __restrict__ counts) {
  __shared__ unsigned int h[256];
  for (int b = threadIdx.x; b < W; b += kB) h[b] = 0u;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * kB;
  for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride) atomicAdd(&h[okey[i]], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < W; b += kB)
    if (h[b]) atomicAdd(&counts[b], (unsigned long long)h[b]);
}

// column 0 of a send row: the token's doc key (u32: IPv4 / 32-bit hashes), or with DOCVAL the
// per-document value doc_val[ids[t]] (the doc's position in the key list sent to its owner)
template <int C, bool DOCVAL>
__global__ void k_route_gather(const int32_t* __restrict__ order, const int64_t* __restrict__ keys,
                               const int32_t* __restrict__ ids, const int32_t* __restrict__ doc_val,
                               const int32_t* __restrict__ word, const int32_t* __restrict__ weight, int64_t n,
                               int32_t* __restrict__ send) {
  const int64_t j = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (j >= n) return;
  const int32_t t = order[j];
  if constexpr (DOCVAL) send[j * C] = doc_val[ids[t]];
  else send[j * C] = (int32_t)(uint32_t)(uint64_t)keys[t];
  send[j * C + 1] = word[t];
  if constexpr (C == 3) send[j * C + 2] = weight[t];
}

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

#define ONI_TRY(x)                          \
  do {                                       \
    const hipError_t e_ = (x);               \
    if (e_ != hipSuccess) return (int)e_;    \
  } while (0)

}  // namespace

// owner_of_id[U]: owner rank of each local document id; ids[n]: document id of every token;
// keys[n]: the documents' u32 keys (int64 storage); word[n]; weight[n] or null.
// Outputs: send[n * (weight ? 3 : 2)] grouped by owner rank (stable), order[n] (token of each
// send slot), counts[W] (tokens per owner). W ≤ 256.
// doc_val (optional, int32 [U]): column 0 carries doc_val[ids[t]] instead of the token's key.
static int route_pack_impl(const int32_t* owner_of_id, const int32_t* ids, const int64_t* keys,
                           const int32_t* doc_val, const int32_t* word, const int32_t* weight, int64_t n, int W,
                           int32_t* send, int32_t* order, int64_t* counts, void* tmp, size_t* tmp_bytes,
                           hipStream_t s) {
  if (n >= (int64_t)1 << 31 || W < 1 || W > 256) return (int)hipErrorInvalidValue;
  int bits = 1;
  while (bits < 8 && ((W - 1) >> bits)) ++bits;
  Arena ar{static_cast<char*>(tmp)};
  uint8_t* okey = ar.take<uint8_t>(n);
  uint8_t* osort = ar.take<uint8_t>(n);
  int32_t* iota = ar.take<int32_t>(n);
  size_t sb = 0;
  ONI_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, sb, okey, osort, iota, order, (int)n, 0, bits, s));
  void* cub = ar.take<char>(sb);
  if (!tmp) {
    *tmp_bytes = ar.used + 256;
    return 0;
  }
  ONI_TRY(hipMemsetAsync(counts, 0, sizeof(int64_t) * W, s));
  if (n == 0) return (int)hipGetLastError();
  k_owner_keys<<<nblk(n), kB, 0, s>>>(owner_of_id, ids, n, okey, iota);
  ONI_TRY(hipcub::DeviceRadixSort::SortPairs(cub, sb, okey, osort, iota, order, (int)n, 0, bits, s));
  const unsigned hb = nblk(n) < 1024u ? nblk(n) : 1024u;
  k_owner_hist<<<hb, kB, 0, s>>>(okey, n, W, reinterpret_cast<unsigned long long*>(counts));
  if (doc_val) {
    if (weight)
      k_route_gather<3, true><<<nblk(n), kB, 0, s>>>(order, keys, ids, doc_val, word, weight, n, send);
    else
      k_route_gather<2, true><<<nblk(n), kB, 0, s>>>(order, keys, ids, doc_val, word, nullptr, n, send);
  } else {
    if (weight)
      k_route_gather<3, false><<<nblk(n), kB, 0, s>>>(order, keys, ids, doc_val, word, weight, n, send);
    else
      k_route_gather<2, false><<<nblk(n), kB, 0, s>>>(order, keys, ids, doc_val, word, nullptr, n, send);
  }
  return (int)hipGetLastError();
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
