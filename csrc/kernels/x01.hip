// X01 payload packing: the per-sweep Δn_wk all-reduce with two 16-bit counts per int32 word.
//
// oni-lda-c reduced K×V doubles over MPI every EM iteration ([U-H]); here the sweep buffer is
// int32 Δn_wk ‖ Δn_k replicas ‖ aux words (oni355/models/gibbs.py). For a realistic vocabulary
// (V ≈ 1e5–1e6 flow words) most words are rare on every rank, and a rare word's
// per-rank value is small: |v| ≤ c_{w,r} (its local token count) whether the sweep sends absolute
// local counts (recount mode) or deltas. Words with max_r c_{w,r} ≤ O = ⌊32767 / W⌋ ("light")
// travel as offset-encoded 16-bit halves e = v + O ∈ [0, 2O] of one int32 word; the ring sum of
// W such halves stays below 2^16, so the low half never carries into the high half and the int32
// sum (two's-complement wrap = u32 arithmetic) decodes exactly as Σe − W·O. Words with
// max_r c_{w,r} ≤ O8 = ⌊127 / W⌋ ("tiny", most of a realistic vocabulary) go as four offset bytes
// per int32 word on the same argument (W bytes of at most 2·O8 sum below 2^8). Heavy rows and the
// tail go as plain int32. Payload = T·KS/4 + L·KS/2 + H·KS + tail words instead of V·KS + tail:
// exact, one collective, and still capturable in the sweep's HIP graph (RCCL has no int8/int16
// reduction on packed lanes).
#include "oni_common.h"

namespace {
constexpr int kB = 256;
inline unsigned nblk(int64_t n) { return (unsigned)((n + kB - 1) / kB > 0 ? (n + kB - 1) / kB : 1); }

__global__ void k_x01_pack(const int32_t* __restrict__ dn, const int32_t* __restrict__ tiny, int64_t T,
                           const int32_t* __restrict__ light, int64_t L, const int32_t* __restrict__ heavy, int64_t H,
                           int KS, int64_t tail_off, int64_t tail_len, int32_t O8, int32_t O,
                           int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  const int quarter = KS >> 2, half = KS >> 1;
  const int64_t nt = T * quarter, nl = L * half, nh = H * KS;
  if (i < nt) {
    const int64_t row = i / quarter;
    const int j = (int)(i - row * quarter);
    const int4 v = *reinterpret_cast<const int4*>(dn + (int64_t)tiny[row] * KS + 4 * j);
    out[i] = (int32_t)((uint32_t)(v.x + O8) | ((uint32_t)(v.y + O8) << 8) | ((uint32_t)(v.z + O8) << 16) |
                       ((uint32_t)(v.w + O8) << 24));
  } else if (i < nt + nl) {
    const int64_t k = i - nt;
    const int64_t row = k / half;
    const int j = (int)(k - row * half);
    const int32_t* src = dn + (int64_t)light[row] * KS + 2 * j;
    const uint32_t a = (uint32_t)(src[0] + O), b = (uint32_t)(src[1] + O);
    out[i] = (int32_t)(a | (b << 16));
  } else if (i < nt + nl + nh) {
    const int64_t k = i - nt - nl;
    const int64_t row = k / KS;
    out[i] = dn[(int64_t)heavy[row] * KS + (k - row * KS)];
  } else if (i < nt + nl + nh + tail_len) {
    out[i] = dn[tail_off + (i - nt - nl - nh)];
  }
}

__global__ void k_x01_unpack(const int32_t* __restrict__ in, const int32_t* __restrict__ tiny, int64_t T,
                             const int32_t* __restrict__ light, int64_t L, const int32_t* __restrict__ heavy, int64_t H,
                             int KS, int64_t tail_off, int64_t tail_len, int32_t WO8, int32_t WO,
                             int32_t* __restrict__ dn) {
  const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  const int quarter = KS >> 2, half = KS >> 1;
  const int64_t nt = T * quarter, nl = L * half, nh = H * KS;
  if (i < nt) {
    const int64_t row = i / quarter;
    const int j = (int)(i - row * quarter);
    const uint32_t v = (uint32_t)in[i];
    *reinterpret_cast<int4*>(dn + (int64_t)tiny[row] * KS + 4 * j) =
        make_int4((int32_t)(v & 0xFFu) - WO8, (int32_t)((v >> 8) & 0xFFu) - WO8, (int32_t)((v >> 16) & 0xFFu) - WO8,
                  (int32_t)(v >> 24) - WO8);
  } else if (i < nt + nl) {
    const int64_t k = i - nt;
    const int64_t row = k / half;
    const int j = (int)(k - row * half);
    const uint32_t v = (uint32_t)in[i];
    int32_t* dst = dn + (int64_t)light[row] * KS + 2 * j;
    dst[0] = (int32_t)(v & 0xFFFFu) - WO;
    dst[1] = (int32_t)(v >> 16) - WO;
  } else if (i < nt + nl + nh) {
    const int64_t k = i - nt - nl;
    const int64_t row = k / KS;
    dn[(int64_t)heavy[row] * KS + (k - row * KS)] = in[i];
  } else if (i < nt + nl + nh + tail_len) {
    dn[tail_off + (i - nt - nl - nh)] = in[i];
  }
}
}  // namespace

// dn: [V·KS | tail] int32; tiny[T] / light[L] / heavy[H]: word ids (disjoint, together all V words);
// out: [T·KS/4 + L·KS/2 + H·KS + tail_len] int32. O8 = ⌊127 / W⌋ and O = ⌊32767 / W⌋ (the caller
// guarantees |v| ≤ O8 on tiny rows and |v| ≤ O on light rows).
ONI_API int oni_x01_pack(const int32_t* dn, const int32_t* tiny, int64_t T, const int32_t* light, int64_t L,
                         const int32_t* heavy, int64_t H, int KS, int64_t tail_off, int64_t tail_len, int O8, int O,
                         int32_t* out, hipStream_t s) {
  if (KS <= 0 || (KS & 3) || O < 0 || O > 32767 || O8 < 0 || O8 > 127) return (int)hipErrorInvalidValue;
  const int64_t n = T * (KS / 4) + L * (KS / 2) + H * KS + tail_len;
  if (n > 0) k_x01_pack<<<nblk(n), kB, 0, s>>>(dn, tiny, T, light, L, heavy, H, KS, tail_off, tail_len, O8, O, out);
  return (int)hipGetLastError();
}

// in: the all-reduced packed buffer; WO8 = W·O8, WO = W·O (the summed offsets). Writes every entry of dn.
ONI_API int oni_x01_unpack(const int32_t* in, const int32_t* tiny, int64_t T, const int32_t* light, int64_t L,
                           const int32_t* heavy, int64_t H, int KS, int64_t tail_off, int64_t tail_len, int WO8,
                           int WO, int32_t* dn, hipStream_t s) {
  if (KS <= 0 || (KS & 3) || WO < 0 || WO > 65535 || WO8 < 0 || WO8 > 255) return (int)hipErrorInvalidValue;
  const int64_t n = T * (KS / 4) + L * (KS / 2) + H * KS + tail_len;
  if (n > 0) k_x01_unpack<<<nblk(n), kB, 0, s>>>(in, tiny, T, light, L, heavy, H, KS, tail_off, tail_len, WO8, WO, dn);
  return (int)hipGetLastError();
}
