// X01 payload packing: the per-sweep Δn_wk all-reduce with two 16-bit counts per int32 word.
//
// oni-lda-c reduced K×V doubles over MPI every EM iteration ([U-H]); here the sweep buffer is
// int32 Δn_wk ‖ Δn_k replicas ‖ aux words (oni355/models/gibbs.py). For a realistic vocabulary
// (V ≈ 1e5–1e6 flow words) most words are rare on every rank, and a rare word's
// per-rank value is small: |v| ≤ c_{w,r} (its local token count) whether the sweep sends absolute
// local counts (recount mode) or deltas. Words with max_r c_{w,r} ≤ O = ⌊32767 / W⌋ ("light")
// travel as offset-encoded 16-bit halves e = v + O ∈ [0, 2O] of one int32 word; the ring sum of
// W such halves stays below 2^16, so the low half never carries into the high half and the int32
// sum (two's-complement wrap = u32 arithmetic) decodes exactly as Σe − W·O. Heavy rows and the
// tail go as plain int32. Payload = L·KS/2 + H·KS + tail words instead of V·KS + tail: exact,
// one collective, and still capturable in the sweep's HIP graph (RCCL has no int16 reduction).
#include "oni_common.h"

namespace {
constexpr int kB = 256;
inline unsigned nblk(int64_t n) { return (unsigned)((n + kB - 1) / kB > 0 ? (n + kB - 1) / kB : 1); }

__global__ void k_x01_pack(const int32_t* __restrict__ dn, const int32_t* __restrict__ light, int64_t L,
                           const int32_t* __restrict__ heavy, int64_t H, int KS, int64_t tail_off, int64_t tail_len,
                           int32_t O, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  const int half = KS >> 1;
  const int64_t nl = L * half, nh = H * KS;
  if (i < nl) {
    const int64_t row = i / half;
    const int j = (int)(i - row * half);
    const int32_t* src = dn + (int64_t)light[row] * KS + 2 * j;
    const uint32_t a = (uint32_t)(src[0] + O), b = (uint32_t)(src[1] + O);
    out[i] = (int32_t)(a | (b << 16));
  } else if (i < nl + nh) {
    const int64_t k = i - nl;
    const int64_t row = k / KS;
    out[i] = dn[(int64_t)heavy[row] * KS + (k - row * KS)];
  } else if (i < nl + nh + tail_len) {
    out[i] = dn[tail_off + (i - nl - nh)];
  }
}

__global__ void k_x01_unpack(const int32_t* __restrict__ in, const int32_t* __restrict__ light, int64_t L,
                             const int32_t* __restrict__ heavy, int64_t H, int KS, int64_t tail_off,
                             int64_t tail_len, int32_t WO, int32_t* __restrict__ dn) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  const int half = KS >> 1;
  const int64_t nl = L * half, nh = H * KS;
  if (i < nl) {
    const int64_t row = i / half;
    const int j = (int)(i - row * half);
    const uint32_t v = (uint32_t)in[i];
    int32_t* dst = dn + (int64_t)light[row] * KS + 2 * j;
    dst[0] = (int32_t)(v & 0xFFFFu) - WO;
    dst[1] = (int32_t)(v >> 16) - WO;
  } else if (i < nl + nh) {
    const int64_t k = i - nl;
    const int64_t row = k / KS;
    dn[(int64_t)heavy[row] * KS + (k - row * KS)] = in[i];
  } else if (i < nl + nh + tail_len) {
    dn[tail_off + (i - nl - nh)] = in[i];
  }
}
}  // namespace

// dn: [V·KS | tail] int32; light[L] / heavy[H]: word ids (disjoint, together all V words);
// out: [L·KS/2 + H·KS + tail_len] int32. O = ⌊32767 / W⌋ (the caller guarantees |v| ≤ O on light rows).
ONI_API int oni_x01_pack(const int32_t* dn, const int32_t* light, int64_t L, const int32_t* heavy, int64_t H, int KS,
                         int64_t tail_off, int64_t tail_len, int O, int32_t* out, hipStream_t s) {
  if (KS <= 0 || (KS & 1) || O < 0 || O > 32767) return (int)hipErrorInvalidValue;
  const int64_t n = L * (KS / 2) + H * KS + tail_len;
  if (n > 0) k_x01_pack<<<nblk(n), kB, 0, s>>>(dn, light, L, heavy, H, KS, tail_off, tail_len, O, out);
  return (int)hipGetLastError();
}

// in: the all-reduced packed buffer; WO = W·O (the summed offset). Writes every entry of dn.
ONI_API int oni_x01_unpack(const int32_t* in, const int32_t* light, int64_t L, const int32_t* heavy, int64_t H, int KS,
                           int64_t tail_off, int64_t tail_len, int WO, int32_t* dn, hipStream_t s) {
  if (KS <= 0 || (KS & 1) || WO < 0 || WO > 65535) return (int)hipErrorInvalidValue;
  const int64_t n = L * (KS / 2) + H * KS + tail_len;
  if (n > 0) k_x01_unpack<<<nblk(n), kB, 0, s>>>(in, light, L, heavy, H, KS, tail_off, tail_len, WO, dn);
  return (int)hipGetLastError();
}
