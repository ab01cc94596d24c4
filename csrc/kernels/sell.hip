// K09 (second half) -- document-term CSR → SELL-S token layout for the sampler.
//
// The reference writes an lda-c corpus (`model.dat`, one line per IP: `M w:c ...`) and ships it
// to MPI ranks. Here the corpus never leaves HBM: the doc-sorted
// (doc, word, count) pairs are cut into chunks of ≤ L tokens (long, power-law IP documents are
// split), chunks are sorted by length and packed S = 64/G to a wave ("slice"),
// and each slice stores its tokens step-major ([step][chunk]) so every sampler step is one
// coalesced 256-B word load + one 64-B topic load per wave.
//
// A token's identity (doc key, position in doc) — not its SELL slot — seeds its RNG draw, so
// the layout can change freely without changing any sample.
#include "oni_common.h"

namespace {

__device__ __forceinline__ int64_t find_pair(const int64_t* __restrict__ tokoff, int64_t lo, int64_t hi, int64_t pos) {
  // last j in [lo, hi) with tokoff[j] <= pos  (pairs of one doc, tokoff ascending)
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (tokoff[mid] <= pos) lo = mid; else hi = mid;
  }
  return lo;
}

__global__ void k_sell_fill(const int32_t* __restrict__ chunk_doc, const int32_t* __restrict__ chunk_pos0,
                            const int32_t* __restrict__ chunk_len, int64_t n_chunks, int S,
                            const int64_t* __restrict__ slice_off, const int64_t* __restrict__ doc_pair_ptr,
                            const int64_t* __restrict__ pair_tokoff, const int32_t* __restrict__ pair_word,
                            const int32_t* __restrict__ pair_cnt, uint32_t* __restrict__ tok_word) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_chunks) return;
  const int d = chunk_doc[i];
  if (d < 0) return;
  const int64_t slice = i / S, lane = i % S;
  const int64_t off = slice_off[slice] + lane;
  const int64_t pos0 = chunk_pos0[i];
  const int len = chunk_len[i];
  int64_t j = find_pair(pair_tokoff, doc_pair_ptr[d], doc_pair_ptr[d + 1], pos0);
  // the current pair's end and word stay in registers: a token of the same pair (most of them) is
  // a store, not two dependent reloads
  int64_t end = pair_tokoff[j] + pair_cnt[j];
  uint32_t w = (uint32_t)pair_word[j];
  for (int s = 0; s < len; ++s) {
    const int64_t pos = pos0 + s;
    while (end <= pos) {
      ++j;
      end = pair_tokoff[j] + pair_cnt[j];
      w = (uint32_t)pair_word[j];
    }
    tok_word[off + (int64_t)s * S] = w;
  }
}

// Move topic assignments between the SELL layout and canonical doc-token order
// (doc-major, word-sorted within doc): dir = 0 gathers SELL → canonical, 1 scatters back.
__global__ void k_sell_perm_z(const int32_t* __restrict__ chunk_doc, const int32_t* __restrict__ chunk_pos0,
                              const int32_t* __restrict__ chunk_len, int64_t n_chunks, int S,
                              const int64_t* __restrict__ slice_off, const int64_t* __restrict__ doc_tok_ptr,
                              uint8_t* __restrict__ tok_z, uint8_t* __restrict__ canon_z, int dir) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_chunks) return;
  const int d = chunk_doc[i];
  if (d < 0) return;
  const int64_t slice = i / S, lane = i % S;
  const int64_t off = slice_off[slice] + lane;
  const int64_t base = doc_tok_ptr[d] + chunk_pos0[i];
  const int len = chunk_len[i];
  for (int s = 0; s < len; ++s) {
    if (dir == 0) canon_z[base + s] = tok_z[off + (int64_t)s * S];
    else tok_z[off + (int64_t)s * S] = canon_z[base + s];
  }
}

}  // namespace

ONI_API int oni_sell_fill(const int32_t* chunk_doc, const int32_t* chunk_pos0, const int32_t* chunk_len,
                          int64_t n_chunks, int S, const int64_t* slice_off, const int64_t* doc_pair_ptr,
                          const int64_t* pair_tokoff, const int32_t* pair_word, const int32_t* pair_cnt,
                          uint32_t* tok_word, hipStream_t s) {
  const unsigned grid = (unsigned)((n_chunks + 255) / 256);
  if (grid == 0) return 0;
  k_sell_fill<<<grid, 256, 0, s>>>(chunk_doc, chunk_pos0, chunk_len, n_chunks, S, slice_off, doc_pair_ptr,
                                   pair_tokoff, pair_word, pair_cnt, tok_word);
  return (int)hipGetLastError();
}

ONI_API int oni_sell_perm_z(const int32_t* chunk_doc, const int32_t* chunk_pos0, const int32_t* chunk_len,
                            int64_t n_chunks, int S, const int64_t* slice_off, const int64_t* doc_tok_ptr,
                            uint8_t* tok_z, uint8_t* canon_z, int dir, hipStream_t s) {
  const unsigned grid = (unsigned)((n_chunks + 255) / 256);
  if (grid == 0) return 0;
  k_sell_perm_z<<<grid, 256, 0, s>>>(chunk_doc, chunk_pos0, chunk_len, n_chunks, S, slice_off, doc_tok_ptr, tok_z,
                                     canon_z, dir);
  return (int)hipGetLastError();
}
