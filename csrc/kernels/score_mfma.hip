// K15 (MFMA variant) -- tiled SDDMM of the post-LDA score on the matrix cores.
//
// Reference behaviour (oni-ml *PostLDA, SURVEY.md §2.2 C24, [U-H]): the score of an event is the
// K-dot θ[doc]·φ[word]. Every distinct (doc, word) pair of the day is scored once (ScorePlan);
// this kernel computes those pair scores as dense 16×16 blocks of Θ_tile · Φ_tileᵀ on
// v_mfma_f32_16x16x4_f32 ("doc-tile × word-union-tile"):
//
//   item = (16 documents, 16 words out of the union of the words those documents use)
//   C[16×16] = Σ_{k-steps} A[16×4] · B[4×16],  A = θ rows of the 16 docs, B = φ rows of the 16 words
//   pair (r, c) of the item  ←  C[r][c], fetched from the accumulator lane by ds_bpermute.
//
// The item plan (which docs form a tile, which words a block, which pairs fall in it, each pair's
// (row, col) byte) is built once per day on the device (oni355/pipeline/common.py tile_plan);
// pairs are stored item-major so the score writes are contiguous.
//
// Numerics: the f32-input MFMA is bit-for-bit a k-ordered fmaf chain starting from 0
// (cdna_hip_programming.md §3 "FP32-input MFMA"), so the NumPy oracle replays it exactly with
// ref.spec.dot_rows_fma. No bf16 rounding: scores near 1e-7 keep their full f32 ordering.
//
// Why MFMA: a per-pair VALU dot re-gathers an 80-B θ row and an 80-B φ row for every pair; a
// 16×16 block gathers 16 + 16 rows once for up to 256 pairs and does the 16×16×K product in
// KS/4 MFMAs (32 cycles each) instead of 256·K lane-FMAs.
#include "oni_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kItemRows = 16;
constexpr int kWavesPerBlock = 4;

template <int KS>
__global__ __launch_bounds__(kWavesPerBlock * 64) void k_tile_score(
    const float* __restrict__ theta, const float* __restrict__ phi, int ks_dyn,
    const int32_t* __restrict__ item_docs,   // [n_items*16] doc row of tile row r (-1: empty row)
    const int32_t* __restrict__ item_words,  // [n_items*16] word row of block column c (-1: empty)
    const int64_t* __restrict__ item_p0,     // [n_items+1] pair range of each item
    const uint8_t* __restrict__ pair_rc,     // [P] (row << 4) | col inside the item
    int64_t n_items, float* __restrict__ ps) {
  const int ks = KS > 0 ? KS : ks_dyn;
  const int lane = oni::lane_id();
  const int r = lane & 15;   // A row / B column held by this lane
  const int kq = lane >> 4;  // k offset inside a 4-deep step
  const int64_t wave_global = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int64_t n_waves = (int64_t)gridDim.x * kWavesPerBlock;
  // the next item's row indices and pair range are fetched one item ahead, so each item waits on
  // one memory round trip (its θ/φ rows) instead of three (indices → rows, range → pair bytes)
  int32_t d_nx = -1, w_nx = -1;
  int64_t p_nx0 = 0, p_nx1 = 0;
  if (wave_global < n_items) {
    d_nx = item_docs[wave_global * kItemRows + r];
    w_nx = item_words[wave_global * kItemRows + r];
    p_nx0 = item_p0[wave_global];
    p_nx1 = item_p0[wave_global + 1];
  }
  for (int64_t it = wave_global; it < n_items; it += n_waves) {
    const int32_t d = d_nx, w = w_nx;
    const int64_t p0 = p_nx0, np = p_nx1 - p_nx0;
    const int64_t nx = it + n_waves;
    if (nx < n_items) {
      d_nx = item_docs[nx * kItemRows + r];
      w_nx = item_words[nx * kItemRows + r];
      p_nx0 = item_p0[nx];
      p_nx1 = item_p0[nx + 1];
    }
    // empty rows/columns read row 0 and multiply by a zero operand: keeps loads unconditional
    const float* ta = theta + (int64_t)(d < 0 ? 0 : d) * ks + kq;
    const float* pb = phi + (int64_t)(w < 0 ? 0 : w) * ks + kq;
    const float ma = d < 0 ? 0.f : 1.f;
    const float mb = w < 0 ? 0.f : 1.f;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (KS > 0) {
      float a[KS > 0 ? KS / 4 : 1], b[KS > 0 ? KS / 4 : 1];
#pragma unroll
      for (int s = 0; s < KS / 4; ++s) {
        a[s] = ta[4 * s] * ma;
        b[s] = pb[4 * s] * mb;
      }
#pragma unroll
      for (int s = 0; s < KS / 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
    } else {
      for (int s = 0; s < ks / 4; ++s)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ta[4 * s] * ma, pb[4 * s] * mb, acc, 0, 0, 0);
    }
    // C[row][col] lives in lane (row >> 2) * 16 + col, register row & 3
    for (int64_t base = 0; base < np; base += 64) {
      const bool ok = base + lane < np;
      const uint32_t rc = ok ? pair_rc[p0 + base + lane] : 0u;
      const int row = (int)(rc >> 4), col = (int)(rc & 15u);
      const int src = ((row >> 2) << 4) | col;
      const float v0 = __shfl(acc[0], src), v1 = __shfl(acc[1], src);
      const float v2 = __shfl(acc[2], src), v3 = __shfl(acc[3], src);
      const int q = row & 3;
      const float v = q == 0 ? v0 : (q == 1 ? v1 : (q == 2 ? v2 : v3));
      if (ok) ps[p0 + base + lane] = v;
    }
  }
}

}  // namespace

ONI_API int oni_tile_score(const float* theta, const float* phi, int KS, const int32_t* item_docs,
                           const int32_t* item_words, const int64_t* item_p0, const uint8_t* pair_rc,
                           int64_t n_items, float* ps, hipStream_t s) {
  if (KS % 4 != 0 || KS <= 0) return (int)hipErrorInvalidValue;
  if (n_items == 0) return 0;
  int64_t blocks = (n_items + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks > 256 * 16) blocks = 256 * 16;
  const unsigned grid = (unsigned)blocks;
#define ONI_T(k_)                                                                                      \
  if (KS == k_) {                                                                                      \
    k_tile_score<k_><<<grid, kWavesPerBlock * 64, 0, s>>>(theta, phi, KS, item_docs, item_words, item_p0, \
                                                         pair_rc, n_items, ps);                        \
    return (int)hipGetLastError();                                                                     \
  }
  ONI_T(20) ONI_T(24) ONI_T(32) ONI_T(52) ONI_T(64) ONI_T(100) ONI_T(104) ONI_T(128)
#undef ONI_T
  k_tile_score<0><<<grid, kWavesPerBlock * 64, 0, s>>>(theta, phi, KS, item_docs, item_words, item_p0, pair_rc,
                                                      n_items, ps);
  return (int)hipGetLastError();
}
