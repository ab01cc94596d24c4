// Host → HBM staging ring: the "decode ‖ H2D ‖ wordify" overlap of SURVEY.md §2.4 P3/P7.
//
// The reference moved a day of events from HDFS into Spark executors and from there into an lda-c
// corpus file copied to every MPI node. Here decoded columns live in host
// memory (mmaped columnar parts or decoder output) and go to HBM once. A plain
// `tensor.to("cuda")` from pageable memory is a synchronous, single-threaded staged copy inside the
// HIP runtime. This ring instead keeps NBUF pinned buffers of `chunk` bytes:
//
//   for each chunk:  wait until buffer b's previous DMA is done (hipEventSynchronize)
//                    fill buffer b from pageable memory with T host threads (memcpy bound)
//                    hipMemcpyAsync(dst + off, buffer b, H2D, stream); record done[b]
//
// so the host copy of chunk i+1 runs while the DMA engine moves chunk i, and the caller returns as
// soon as the last copy is queued: kernels the caller launches next on the same stream (wordify,
// quantile keys) are ordered after the copies by the stream, while the CPU goes on decoding the
// next part. Ring state persists across calls, so consecutive columns pipeline as one stream of
// chunks. Pure host code: no device kernel is involved.
//
// Measured (profiles/r1_h2d_staging.jsonl): the H2D of a 12.5M-flow day is PCIe-link bound on every
// path (≈55 GB/s); ROCm's pageable copy already reaches it, the ring reaches 52 GB/s at 32 MB x 16
// threads, so io/staging.py defaults to the plain copy and keeps the ring / registered paths as
// options.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr int kMaxBuf = 8;

struct Stager {
  size_t chunk = 0;
  int nbuf = 0;
  int threads = 1;
  int next = 0;
  void* buf[kMaxBuf] = {};
  hipEvent_t done[kMaxBuf] = {};
  bool pending[kMaxBuf] = {};
  uint64_t bytes_staged = 0;
  uint64_t chunks_staged = 0;
};

void par_memcpy(void* dst, const void* src, size_t n, int threads) {
  // ≥ 1 MiB per thread, else the thread start costs more than the copy
  const size_t min_per = size_t(1) << 20;
  int t = (int)std::min<size_t>((size_t)std::max(threads, 1), std::max<size_t>(n / min_per, 1));
  if (t <= 1) {
    std::memcpy(dst, src, n);
    return;
  }
  const size_t per = (n + t - 1) / t;
  std::vector<std::thread> ws;
  ws.reserve(t - 1);
  for (int i = 1; i < t; ++i) {
    const size_t lo = std::min(n, per * i), hi = std::min(n, per * (i + 1));
    if (hi > lo)
      ws.emplace_back([=] { std::memcpy((char*)dst + lo, (const char*)src + lo, hi - lo); });
  }
  std::memcpy(dst, src, std::min(n, per));
  for (auto& w : ws) w.join();
}

// Copy-engine-free upload: the CUs pull page-locked host memory over PCIe. A bulk hipMemcpyAsync
// occupies the DMA engine, and every later small transfer in either direction -- a histogram
// read-back, a .item(), a count upload before an all-to-all -- queues behind it
// (bench/overlap_probe.py: a 32 KB D2H waits 11 ms behind a 550 MB upload; kernels, graph
// replays, D2D copies and RCCL collectives do not). Pulling with a few workgroups leaves the DMA
// engine to those small transfers. 4 × 16 B loads per thread in flight; stores bypass L2 residency.
constexpr int kPullThreads = 256;
constexpr int kPullUnroll = 4;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kPullThreads) void k_pull(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                       int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * kPullThreads * kPullUnroll;
  for (int64_t base = (int64_t)blockIdx.x * kPullThreads * kPullUnroll + threadIdx.x; base < n16; base += stride) {
    u32x4 v[kPullUnroll];
#pragma unroll
    for (int u = 0; u < kPullUnroll; ++u) {
      const int64_t i = base + (int64_t)u * kPullThreads;
      if (i < n16) v[u] = src[i];
    }
#pragma unroll
    for (int u = 0; u < kPullUnroll; ++u) {
      const int64_t i = base + (int64_t)u * kPullThreads;
      if (i < n16) __builtin_nontemporal_store(v[u], dst + i);
    }
  }
}

__global__ void k_pull_tail(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int n) {
  if ((int)threadIdx.x < n) dst[threadIdx.x] = src[threadIdx.x];
}

// Device → page-locked host words written by a kernel (the read-back twin of k_pull): small
// values the host polls during a run (the sampler's changed-token count) do not wait behind a
// bulk upload on the DMA engine. One vector store per word, then a system-scope fence.
__global__ void k_push_words(const uint32_t* __restrict__ src, uint32_t* dst, int n) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i < n) {
    __builtin_nontemporal_store(src[i], dst + i);
    __threadfence_system();
  }
}

}  // namespace

extern "C" {

// Copy `words` 32-bit words from device `src` into page-locked host memory `host_dst` on `stream`
// with a kernel. The host reads them after an event recorded behind this call has completed.
// hipErrorInvalidValue when `host_dst` is not device-visible pinned memory.
int oni_d2h_push(const void* src, void* host_dst, int64_t words, hipStream_t stream) {
  if (words <= 0) return 0;
  if (words > (int64_t)1 << 24) return (int)hipErrorInvalidValue;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, host_dst, 0) != hipSuccess || d == nullptr) {
    (void)hipGetLastError();
    return (int)hipErrorInvalidValue;
  }
  const int n = (int)words;
  k_push_words<<<(n + 255) / 256, 256, 0, stream>>>(static_cast<const uint32_t*>(src), static_cast<uint32_t*>(d), n);
  return (int)hipGetLastError();
}

// Upload `bytes` from page-locked host memory `src` (hipHostMalloc / torch pin_memory) to `dst` on
// `stream` with `blocks` workgroups (0 → 64) instead of the DMA engine. Asynchronous like
// hipMemcpyAsync. Returns hipErrorInvalidValue when `src` is not device-visible pinned memory (the
// caller then uses hipMemcpyAsync).
int oni_h2d_pull(const void* src, void* dst, int64_t bytes, int blocks, hipStream_t stream) {
  if (bytes <= 0) return 0;
  void* dsrc = nullptr;
  if (hipHostGetDevicePointer(&dsrc, const_cast<void*>(src), 0) != hipSuccess || dsrc == nullptr) {
    (void)hipGetLastError();
    return (int)hipErrorInvalidValue;
  }
  const bool aligned = ((uintptr_t)dsrc % 16 == 0) && ((uintptr_t)dst % 16 == 0);
  if (!aligned && bytes > 4096) return (int)hipErrorInvalidValue;  // caller falls back to the DMA copy
  const int64_t n16 = aligned ? bytes / 16 : 0;
  const int64_t done = n16 * 16;
  if (n16 > 0) {
    const int64_t per_block = (int64_t)kPullThreads * kPullUnroll;
    const int64_t need = (n16 + per_block - 1) / per_block;
    const int grid = (int)std::min<int64_t>(need, blocks > 0 ? blocks : 64);
    k_pull<<<grid, kPullThreads, 0, stream>>>(static_cast<const u32x4*>(dsrc), static_cast<u32x4*>(dst), n16);
  }
  for (int64_t off = done; off < bytes; off += 256) {  // remainder (< 16 B, or a small unaligned buffer)
    const int n = (int)std::min<int64_t>(256, bytes - off);
    k_pull_tail<<<1, 256, 0, stream>>>(static_cast<const uint8_t*>(dsrc) + off, static_cast<uint8_t*>(dst) + off, n);
  }
  return (int)hipGetLastError();
}

// Create a ring of `nbuf` pinned buffers of `chunk_bytes`; `threads` host threads fill each one.
// Returns 0 on success, the hipError otherwise; *out receives the handle.
int oni_stager_create(int64_t chunk_bytes, int nbuf, int threads, void** out) {
  if (chunk_bytes <= 0 || nbuf < 2 || nbuf > kMaxBuf || out == nullptr) return (int)hipErrorInvalidValue;
  auto* s = new Stager();
  s->chunk = (size_t)chunk_bytes;
  s->nbuf = nbuf;
  s->threads = std::max(threads, 1);
  for (int i = 0; i < nbuf; ++i) {
    hipError_t e = hipHostMalloc(&s->buf[i], s->chunk, hipHostMallocDefault);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s->done[i], hipEventDisableTiming);
    if (e != hipSuccess) {
      for (int j = 0; j <= i; ++j) {
        if (s->buf[j]) (void)hipHostFree(s->buf[j]);
        if (s->done[j]) (void)hipEventDestroy(s->done[j]);
      }
      delete s;
      return (int)e;
    }
  }
  *out = s;
  return 0;
}

// Queue `bytes` from pageable `src` to device `dst` on `stream` through the ring. Returns once the
// last chunk is queued (not when it has landed): order later work on `stream`, or call
// oni_stager_sync, before reading `dst` elsewhere. `src` is consumed synchronously (copied into
// pinned buffers before this call returns), so the caller may free or overwrite it at once.
int oni_stager_upload(void* handle, const void* src, void* dst, int64_t bytes, hipStream_t stream) {
  auto* s = static_cast<Stager*>(handle);
  if (s == nullptr || bytes < 0 || (bytes > 0 && (src == nullptr || dst == nullptr)))
    return (int)hipErrorInvalidValue;
  size_t off = 0;
  const size_t n = (size_t)bytes;
  while (off < n) {
    const int b = s->next;
    if (s->pending[b]) {
      hipError_t e = hipEventSynchronize(s->done[b]);
      if (e != hipSuccess) return (int)e;
      s->pending[b] = false;
    }
    const size_t len = std::min(s->chunk, n - off);
    par_memcpy(s->buf[b], (const char*)src + off, len, s->threads);
    hipError_t e = hipMemcpyAsync((char*)dst + off, s->buf[b], len, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) e = hipEventRecord(s->done[b], stream);
    if (e != hipSuccess) return (int)e;
    s->pending[b] = true;
    s->next = (b + 1) % s->nbuf;
    off += len;
    s->bytes_staged += len;
    s->chunks_staged += 1;
  }
  return 0;
}

// Wait for every queued chunk (the ring's buffers are then free).
int oni_stager_sync(void* handle) {
  auto* s = static_cast<Stager*>(handle);
  if (s == nullptr) return (int)hipErrorInvalidValue;
  for (int b = 0; b < s->nbuf; ++b) {
    if (s->pending[b]) {
      hipError_t e = hipEventSynchronize(s->done[b]);
      if (e != hipSuccess) return (int)e;
      s->pending[b] = false;
    }
  }
  return 0;
}

// Bytes and chunks moved through the ring since creation.
int oni_stager_stats(void* handle, int64_t* out2) {
  auto* s = static_cast<Stager*>(handle);
  if (s == nullptr || out2 == nullptr) return (int)hipErrorInvalidValue;
  out2[0] = (int64_t)s->bytes_staged;
  out2[1] = (int64_t)s->chunks_staged;
  return 0;
}

// Zero-copy alternative to the ring: pin `src` in place (hipHostRegister), DMA it straight to
// `dst` on `stream`, wait, unpin. Synchronous (the pages must stay pinned until the DMA is done).
int oni_h2d_registered(const void* src, void* dst, int64_t bytes, hipStream_t stream) {
  if (bytes <= 0) return 0;
  hipError_t e = hipHostRegister(const_cast<void*>(src), (size_t)bytes, hipHostRegisterDefault);
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  hipError_t u = hipHostUnregister(const_cast<void*>(src));
  return (int)(e != hipSuccess ? e : u);
}

int oni_stager_destroy(void* handle) {
  auto* s = static_cast<Stager*>(handle);
  if (s == nullptr) return 0;
  int rc = oni_stager_sync(handle);
  for (int b = 0; b < s->nbuf; ++b) {
    (void)hipEventDestroy(s->done[b]);
    (void)hipHostFree(s->buf[b]);
  }
  delete s;
  return rc;
}

}  // extern "C"
