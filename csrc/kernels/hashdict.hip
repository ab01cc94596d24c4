// K08 fast path -- dictionary encoding by hashing when the distinct keys are few.
//
// dict_encode (corpus.hip) sorts all n keys (a full radix sort of 25M keys + a 25M-element random
// scatter for the inverse: ~1.4 ms per dictionary on the 12.5M-flow day). A day has only ~6k
// distinct flow words and ~370k IP documents, so here every key is inserted into an open-
// addressing table (64-bit keys, linear probing) after a block-local LDS de-duplication -- a
// block touches the global table once per distinct key it saw, and a key already present costs a
// plain load, not an atomic -- then only the V distinct keys are sorted, their ranks written back
// into the table, and every key looks up its rank. Two streaming passes over the keys instead of
// four sort passes + a scatter; the outputs are identical to the sort path (sorted unique keys,
// id = rank). Too many distinct keys for the table (or a pathological probe chain) raises a flag
// and the caller falls back to the sort path.
#include <hipcub/hipcub.hpp>

#include "oni_common.h"

namespace {

constexpr int kB = 256;
constexpr uint64_t kEmpty = ~0ull;  // never a key: word keys < 2^62, document keys < 2^32 (the build rejects nothing: a key
                                    // equal to it would be dropped, so callers pass keys < 2^63)
constexpr int kLSlots = 2048;       // block-local LDS set (16 KB)
constexpr int kLProbe = 8;          // LDS probe limit
constexpr int kPerThread = 16;      // keys per thread in the insert pass
constexpr int kMaxProbe = 4096;

inline unsigned nblk(int64_t n, int64_t per) { return (unsigned)((n + per - 1) / per > 0 ? (n + per - 1) / per : 1); }

__device__ __forceinline__ uint32_t mix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return (uint32_t)k;
}

__global__ void k_hd_fill(uint64_t* __restrict__ tab, int32_t* __restrict__ val, int64_t m) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (i < m) {
    tab[i] = kEmpty;
    val[i] = -1;
  }
}

// insert: LDS de-dup, then the block's first sighting of a key probes the global table
__global__ __launch_bounds__(kB) void k_hd_insert(const uint64_t* __restrict__ keys, int64_t n, uint64_t* tab,
                                                  uint32_t mask, uint32_t* __restrict__ n_unique,
                                                  uint32_t* __restrict__ overflow) {
  __shared__ unsigned long long ls[kLSlots];
  for (int s = threadIdx.x; s < kLSlots; s += kB) ls[s] = kEmpty;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kB * kPerThread;
  for (int r = 0; r < kPerThread; ++r) {
    const int64_t i = base + (int64_t)r * kB + threadIdx.x;
    if (i >= n) break;
    const unsigned long long k = keys[i];
    bool fresh = true;
    uint32_t h = mix(k) & (kLSlots - 1);
    // short local probe chains: with more distinct keys than the LDS set holds (documents) the
    // set fills up, and a key not found nearby simply goes to the global table
    for (int p = 0; p < kLProbe; ++p) {
      const unsigned long long old = atomicCAS(&ls[h], (unsigned long long)kEmpty, k);
      if (old == kEmpty) break;           // first sighting in this block
      if (old == k) {                     // seen by this block already
        fresh = false;
        break;
      }
      h = (h + 1) & (kLSlots - 1);
    }
    if (!fresh) continue;
    uint32_t g = mix(k) & mask;
    int p = 0;
    for (; p < kMaxProbe; ++p) {
      const unsigned long long cur = __hip_atomic_load(reinterpret_cast<unsigned long long*>(tab) + g,
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == k) break;
      if (cur == kEmpty) {
        const unsigned long long old =
            atomicCAS(reinterpret_cast<unsigned long long*>(tab) + g, (unsigned long long)kEmpty, k);
        if (old == kEmpty) {
          atomicAdd(n_unique, 1u);
          break;
        }
        if (old == k) break;
      }
      g = (g + 1) & mask;
      // a table past half full is abandoned anyway: stop probing instead of walking long chains
      if ((p & 63) == 63 && __hip_atomic_load(n_unique, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > (mask >> 1)) {
        p = kMaxProbe;
        break;
      }
    }
    if (p == kMaxProbe) atomicOr(overflow, 1u);
  }
}

// occupied slots → unsorted unique keys
// one counter atomic per wave (ballot + prefix popcount): a per-slot atomic on the one counter
// serialised 170k times at a realistic vocabulary (0.69 ms); the order is irrelevant (sorted next)
__global__ void k_hd_compact(const uint64_t* __restrict__ tab, int64_t m, uint64_t* __restrict__ uniq,
                             uint32_t* __restrict__ cnt, uint32_t cap) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  const uint64_t k = i < m ? tab[i] : kEmpty;
  const bool keep = k != kEmpty;
  const uint64_t b = __ballot(keep);
  if (b == 0ull) return;
  const int lane = oni::lane_id();
  const int leader = __ffsll((unsigned long long)b) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(cnt, (uint32_t)__popcll(b));
  base = (uint32_t)__shfl((int)base, leader);
  if (keep) {
    const uint32_t at = base + (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
    if (at < cap) uniq[at] = k;  // beyond cap the caller falls back to the sort path
  }
}

__device__ __forceinline__ uint32_t find(const uint64_t* __restrict__ tab, uint32_t mask, uint64_t k) {
  uint32_t g = mix(k) & mask;
  for (int p = 0; p < kMaxProbe; ++p) {
    const uint64_t cur = tab[g];
    if (cur == k || cur == kEmpty) return g;
    g = (g + 1) & mask;
  }
  return g;
}

// rank of every sorted unique key → its slot's value
__global__ void k_hd_rank2(const uint64_t* __restrict__ sorted, int64_t nu, const uint64_t* __restrict__ tab,
                           uint32_t mask, int32_t* __restrict__ val) {
  const int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (r < nu) val[find(tab, mask, sorted[r])] = (int32_t)r;
}

// rank r of every sorted unique key into a compact table (built after the host read nu): a table
// of ≥ 4·nu slots that the L2 holds (32k slots = 384 KB at the 5.7k-word default day) instead of
// the 48-MB build table whose random probes miss to the MALL
__global__ void k_hd_small_insert(const uint64_t* __restrict__ sorted, int64_t nu, uint64_t* tab, uint32_t mask,
                                  int32_t* __restrict__ val) {
  const int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x;
  if (r >= nu) return;
  const unsigned long long k = sorted[r];
  uint32_t g = mix(k) & mask;
  for (int p = 0; p < kMaxProbe; ++p) {  // ≤ 1/4 full, distinct keys: a free slot is always near
    const unsigned long long old =
        atomicCAS(reinterpret_cast<unsigned long long*>(tab) + g, (unsigned long long)kEmpty, k);
    if (old == kEmpty) {
      val[g] = (int32_t)r;
      return;
    }
    g = (g + 1) & mask;
  }
}

// four keys per lane (coalesced at stride kB): their key → slot → value chains overlap instead of
// one chain of three dependent loads per lane
constexpr int kLookupPer = 4;

__global__ void k_hd_lookup(const uint64_t* __restrict__ keys, int64_t n, const uint64_t* __restrict__ tab,
                            uint32_t mask, const int32_t* __restrict__ val, int32_t* __restrict__ ids) {
  const int64_t base = (int64_t)blockIdx.x * kB * kLookupPer + threadIdx.x;
  uint64_t k[kLookupPer];
  uint32_t g[kLookupPer];
#pragma unroll
  for (int j = 0; j < kLookupPer; ++j) {
    const int64_t i = base + (int64_t)j * kB;
    k[j] = i < n ? keys[i] : 0ull;
  }
#pragma unroll
  for (int j = 0; j < kLookupPer; ++j) g[j] = find(tab, mask, k[j]);
#pragma unroll
  for (int j = 0; j < kLookupPer; ++j) {
    const int64_t i = base + (int64_t)j * kB;
    if (i < n) ids[i] = val[g[j]];
  }
}

#define ONI_TRY(x)                          \
  do {                                       \
    const hipError_t e_ = (x);               \
    if (e_ != hipSuccess) return (int)e_;    \
  } while (0)


}  // namespace

// Phase A: table build into caller buffers tab[M] u64, val[M] i32, unsorted[M/2 + 1] u64 (M =
// table_slots, a power of two). status[3] (device) ← [0] distinct keys, [1] overflow flag,
// [2] compacted count. The caller reads status: when the flag is set or [0] > M/2 the table is
// unusable (use the sort path). Keys must be < 2^63 (~0 marks an empty slot).
ONI_API int oni_hashdict_build(const uint64_t* keys, int64_t n, int64_t table_slots, void* tab_v, void* val_v,
                               void* unsorted_v, uint32_t* status, hipStream_t s) {
  if (n >= (int64_t)1 << 31 || table_slots < 2 || (table_slots & (table_slots - 1)) || table_slots > ((int64_t)1 << 30))
    return (int)hipErrorInvalidValue;
  auto* tab = static_cast<uint64_t*>(tab_v);
  auto* val = static_cast<int32_t*>(val_v);
  auto* unsorted = static_cast<uint64_t*>(unsorted_v);
  const uint32_t mask = (uint32_t)(table_slots - 1);
  ONI_TRY(hipMemsetAsync(status, 0, 3 * sizeof(uint32_t), s));
  if (n == 0) return (int)hipGetLastError();
  k_hd_fill<<<nblk(table_slots, kB), kB, 0, s>>>(tab, val, table_slots);
  k_hd_insert<<<nblk(n, (int64_t)kB * kPerThread), kB, 0, s>>>(keys, n, tab, mask, status, status + 1);
  k_hd_compact<<<nblk(table_slots, kB), kB, 0, s>>>(tab, table_slots, unsorted, status + 2,
                                                     (uint32_t)(table_slots / 2 + 1));
  return (int)hipGetLastError();
}

// Phase B (after the caller read nu = status[0] ≤ M/2, no overflow): sort the nu distinct keys
// into uniq, rank them in the table, look every key up → ids[n]. tmp: hipCUB scratch (two-phase).
ONI_API int oni_hashdict_finish(const uint64_t* keys, int64_t n, int key_bits, int64_t table_slots, const void* tab_v,
                                void* val_v, const void* unsorted_v, int64_t nu, uint64_t* uniq, int32_t* ids,
                                void* tmp, size_t* tmp_bytes, hipStream_t s) {
  const uint32_t mask = (uint32_t)(table_slots - 1);
  auto* tab = static_cast<const uint64_t*>(tab_v);
  auto* val = static_cast<int32_t*>(val_v);
  auto* unsorted = static_cast<const uint64_t*>(unsorted_v);
  size_t sb = 0;
  ONI_TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, sb, unsorted, uniq, (int)(nu > 0 ? nu : 1), 0, key_bits, s));
  // compact lookup table of ≥ 4·nu slots when that is smaller than the build table
  int64_t m2 = 1024;
  while (m2 < 4 * nu) m2 <<= 1;
  const bool compact = m2 < table_slots;
  const size_t sb_al = (sb + 255) & ~size_t(255);
  if (!tmp) {
    *tmp_bytes = sb_al + (compact ? (size_t)m2 * 12 : 0) + 256;
    return 0;
  }
  if (n == 0 || nu == 0) return (int)hipGetLastError();
  ONI_TRY(hipcub::DeviceRadixSort::SortKeys(tmp, sb, unsorted, uniq, (int)nu, 0, key_bits, s));
  if (compact) {
    auto* tab2 = reinterpret_cast<uint64_t*>(static_cast<char*>(tmp) + sb_al);
    auto* val2 = reinterpret_cast<int32_t*>(tab2 + m2);
    const uint32_t mask2 = (uint32_t)(m2 - 1);
    k_hd_fill<<<nblk(m2, kB), kB, 0, s>>>(tab2, val2, m2);
    k_hd_small_insert<<<nblk(nu, kB), kB, 0, s>>>(uniq, nu, tab2, mask2, val2);
    k_hd_lookup<<<nblk(n, (int64_t)kB * kLookupPer), kB, 0, s>>>(keys, n, tab2, mask2, val2, ids);
  } else {
    k_hd_rank2<<<nblk(nu, kB), kB, 0, s>>>(uniq, nu, tab, mask, val);
    k_hd_lookup<<<nblk(n, (int64_t)kB * kLookupPer), kB, 0, s>>>(keys, n, tab, mask, val, ids);
  }
  return (int)hipGetLastError();
}
