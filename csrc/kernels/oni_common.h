// oni355 -- shared device helpers for the CDNA4 (gfx950) kernels.
//
// Everything here is written for wave64 / gfx950 only: no CUDA shims, no dual paths.
// Numerics are pinned (the build uses -ffp-contract=off) so that the NumPy oracle in
// oni355/ref/spec.py can replay the sampler and the featurizers bit-for-bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ONI_API extern "C" __attribute__((visibility("default")))

namespace oni {

constexpr int kWave = 64;
constexpr uint32_t kPadWord = 0xFFFFFFFFu;   // SELL padding token

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 counter RNG (Salmon et al., SC'11). Keyed by the run seed; the counter encodes
// (position-in-document / 4, document key, sweep, stream tag), so every draw is a pure function
// of (seed, sweep, doc, pos): independent of GPU count, chunking, SELL layout and scheduling.
// ---------------------------------------------------------------------------------------------
struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32->64 multiply per product (v_mad_u64_u32) instead of separate lo / hi halves
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Philox2x32-10: two words per counter (pos, doc key) under key k -- half the multiplies of the
// 4x32 generator where a draw needs two words.
__device__ __forceinline__ void philox2x32_10(uint32_t& c0, uint32_t& c1, uint32_t k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p = (uint64_t)0xD256D193u * c0;
    const uint32_t hi = (uint32_t)(p >> 32), lo = (uint32_t)p;
    c0 = hi ^ k ^ c1;
    c1 = lo;
    k += 0x9E3779B9u;
  }
}

__device__ __forceinline__ uint32_t pick4(const U4& r, uint32_t i) {
  return i == 0 ? r.x : (i == 1 ? r.y : (i == 2 ? r.z : r.w));
}

// 32-bit integer mixer (lowbias32, C. Wellons): the seed-free initial topic of a word.
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// 24-bit uniform in [0,1): exact in f32 on both sides (GPU and NumPy oracle).
__device__ __forceinline__ float u01(uint32_t r) { return (float)(r >> 8) * 5.9604644775390625e-08f; }

// Order-preserving f32 -> u32 map (radix-select / histogram keys).
__device__ __forceinline__ uint32_t f32_key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_f32(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// wave-wide lane index / ballot helpers (64-bit masks on CDNA)
__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Grid-stride helper sized for 256 CUs: callers launch min(ceil(n/256), 256*8) blocks.
__host__ __forceinline__ unsigned grid_for(int64_t n, int block = 256, int cap = 2048) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

}  // namespace oni
