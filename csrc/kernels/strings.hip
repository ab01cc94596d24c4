// K04/K06/K07 -- GPU string featurization for DNS query names, proxy hosts/URIs/user agents.
//
// Reference behaviour (oni-ml DNSWordCreation / DomainProcessor.extractDomainInfo / Entropy /
// TopDomains, ProxyWordCreation; SURVEY.md §2.2 C17/C18, §2.8, [U-M]): split a name into
// subdomain / registered domain / public suffix (table-driven PSL rules, oni355/ref/psl.py),
// flag user-domain and
// top-1M membership, measure subdomain length, Shannon entropy and dot count.
//
// Layout: N strings as int64 offsets [N+1] + UTF-8 bytes (the columnar store's native form).
// One lane per string; bytes are read straight from global memory (names average ~25 B, so a
// wave's 64 names span a few KB that stay in L1/L2). Entropy uses a per-lane 64-bin character
// histogram in LDS (u8 counts; names are ≤ 253 B) and host-built f32 tables of c·log2(c) and
// log2(n), so the GPU and the NumPy oracle agree bit-for-bit. Set membership (top-1M registered
// domains) is an open-addressing table of 64-bit FNV-1a hashes, built on the host once.
#include "oni_common.h"

namespace {

constexpr int kBins = 64;
constexpr uint64_t kFnvOff = 1469598103934665603ull, kFnvPrime = 1099511628211ull;

__device__ __forceinline__ uint8_t lower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c; }

// character class for the entropy histogram: a-z 0..25, 0-9 26..35, '-' 36, '_' 37, '.' 38,
// other bytes folded into 39..63 by value
__device__ __forceinline__ int cbin(uint8_t c) {
  if (c >= 'a' && c <= 'z') return c - 'a';
  if (c >= '0' && c <= '9') return 26 + (c - '0');
  if (c == '-') return 36;
  if (c == '_') return 37;
  if (c == '.') return 38;
  return 39 + (c % 25);
}

__device__ __forceinline__ uint64_t fnv_range(const uint8_t* p, int64_t a, int64_t b) {
  uint64_t h = kFnvOff;
  for (int64_t i = a; i < b; ++i) h = (h ^ lower(p[i])) * kFnvPrime;
  return h;
}

__device__ __forceinline__ bool set_probe(const uint64_t* __restrict__ tab, uint64_t mask, uint64_t h) {
  if (!tab) return false;
  if (h == 0) h = 1;
  uint64_t i = (h ^ (h >> 29)) & mask;
  for (int n = 0; n <= (int)mask && n < 4096; ++n) {
    const uint64_t v = tab[i];
    if (v == h) return true;
    if (v == 0) return false;
    i = (i + 1) & mask;
  }
  return false;
}

// H of an n-byte histogram (n ≥ 1), bins summed in index order
__device__ __forceinline__ float entropy_of_hist(const uint8_t* h, int n, const float* __restrict__ clogc,
                                                 const float* __restrict__ lg) {
  float s = 0.f;
  for (int k = 0; k < kBins; ++k) s = s + clogc[h[k]];
  return lg[n < 255 ? n : 255] - s / (float)n;
}

// Shannon entropy (bits) of bytes [a, b) with the exact-table formulation:
//   H = lg[n] - (Σ_bins clogc[c_bin]) / n,    clogc[c] = c·log2(c), lg[n] = log2(n)  (f32 tables)
__device__ float entropy_range(const uint8_t* __restrict__ p, int64_t a, int64_t b, uint8_t* h,
                               const float* __restrict__ clogc, const float* __restrict__ lg) {
  const int n = (int)(b - a);
  if (n <= 0) return 0.f;
  for (int k = 0; k < kBins; ++k) h[k] = 0;
  for (int64_t i = a; i < b; ++i) {
    const int k = cbin(lower(p[i]));
    h[k] = (uint8_t)(h[k] + 1);
  }
  return entropy_of_hist(h, n, clogc, lg);
}

struct DomainOut {
  uint64_t* reg_hash;   // FNV-1a of the registered domain (label.suffix)
  uint8_t* top;         // 2 user domain, 1 top-1M, 0 other
  int32_t* sub_len;     // subdomain length in bytes
  float* sub_ent;       // subdomain entropy (bits)
  int32_t* periods;     // '.' count of the (trailing-dot-stripped) name
  int32_t* sub_off;     // [N][2] subdomain / registered-domain start offsets (relative)
};

// Public-suffix rules (oni355/ref/psl.py): two open-addressing FNV-1a sets, exact / wildcard rules
// (the latter stored as "*.rest") and exceptions (without the '!').
struct Psl {
  const uint64_t* rules;
  uint64_t rules_mask;
  const uint64_t* exc;
  uint64_t exc_mask;
  int max_labels;  // ≤ kMaxLabels
};
constexpr int kMaxLabels = 6;

__device__ __forceinline__ uint64_t fnv_cont(uint64_t h, const uint8_t* p, int64_t a, int64_t b) {
  for (int64_t i = a; i < b; ++i) h = (h ^ lower(p[i])) * kFnvPrime;
  return h;
}

// Start of the registered domain of [a, b): public suffix by the PSL algorithm (longest deciding
// suffix; exception → one label shorter; no rule → last label), plus one more label.
// dots[j] = position of the (j+1)-th '.' from the right (at most max_labels of them, nd found).
__device__ int64_t registered_start(const uint8_t* __restrict__ p, int64_t a, int64_t b, const int64_t* dots, int nd,
                                    const Psl& psl) {
  const int nlab = b > a ? nd + 1 : 0;
  // FNV state after "*." (wildcard rules)
  const uint64_t wild0 = (((kFnvOff ^ (uint64_t)'*') * kFnvPrime) ^ (uint64_t)'.') * kFnvPrime;
  int ps = 1;
  const int kmax = nlab < psl.max_labels ? nlab : psl.max_labels;
  for (int k = kmax; k >= 1; --k) {
    const int64_t sk = k <= nd ? dots[k - 1] + 1 : a;
    const uint64_t h = fnv_range(p, sk, b);
    if (set_probe(psl.exc, psl.exc_mask, h)) {
      ps = k - 1;
      break;
    }
    bool hit = set_probe(psl.rules, psl.rules_mask, h);
    if (!hit && k >= 2) {
      const int64_t sk1 = (k - 1) <= nd ? dots[k - 2] + 1 : a;
      hit = set_probe(psl.rules, psl.rules_mask, fnv_cont(wild0, p, sk1, b));
    }
    if (hit) {
      ps = k;
      break;
    }
  }
  if (nlab <= ps) return a;
  return ps + 1 <= nd ? dots[ps] + 1 : a;
}

__global__ __launch_bounds__(256) void k_domain_features(const int64_t* __restrict__ off, const uint8_t* __restrict__ p,
                                                         int64_t n, const uint64_t* __restrict__ top_tab,
                                                         uint64_t top_mask, uint64_t user_hash, int user_is_label,
                                                         const float* __restrict__ clogc, const float* __restrict__ lg,
                                                         Psl psl, DomainOut o) {
  __shared__ uint8_t hist[256][kBins];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t a = off[i];
    int64_t b = off[i + 1];
    while (b > a && p[b - 1] == '.') --b;  // trailing root dot
    // dot positions from the right (as many as the suffix rules can look at) + the total count
    int64_t dots[kMaxLabels];
    int nd = 0, per = 0;
    for (int64_t j = b - 1; j >= a; --j)
      if (p[j] == '.') {
        ++per;
        if (nd < psl.max_labels) dots[nd++] = j;
      }
    const int64_t reg = registered_start(p, a, b, dots, nd, psl);  // start of registered domain
    const int64_t sub_end = reg > a ? reg - 1 : a;  // subdomain = [a, reg-1)
    const uint64_t rh = fnv_range(p, reg, b);
    // registered label only (for USER_DOMAIN given as a bare label, e.g. "intel")
    int64_t lab_end = reg;
    while (lab_end < b && p[lab_end] != '.') ++lab_end;
    const uint64_t lh = fnv_range(p, reg, lab_end);
    uint8_t top = 0;
    if (user_hash != 0 && (user_is_label ? lh == user_hash : rh == user_hash)) top = 2;
    else if (set_probe(top_tab, top_mask, rh)) top = 1;
    o.reg_hash[i] = rh;
    o.top[i] = top;
    o.sub_len[i] = (int32_t)(sub_end - a);
    o.periods[i] = per;
    o.sub_ent[i] = entropy_range(p, a, sub_end, hist[threadIdx.x], clogc, lg);
    if (o.sub_off) {
      o.sub_off[2 * i] = 0;
      o.sub_off[2 * i + 1] = (int32_t)(reg - a);
    }
  }
}

// Generic per-string features: FNV-1a hash (lowercased), length, entropy.
__global__ __launch_bounds__(256) void k_string_features(const int64_t* __restrict__ off, const uint8_t* __restrict__ p,
                                                         int64_t n, const float* __restrict__ clogc,
                                                         const float* __restrict__ lg, uint64_t* __restrict__ hash,
                                                         int32_t* __restrict__ len, float* __restrict__ ent) {
  __shared__ uint8_t hist[256][kBins];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // one pass over 4-B aligned words (the word holding a string's last byte never leaves the
  // 4-B-aligned allocation): the hash and the histogram share each load, a quarter of the
  // load instructions of two byte-wise passes
  const bool al = (reinterpret_cast<uintptr_t>(p) & 3u) == 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t a = off[i], b = off[i + 1];
    if (len) len[i] = (int32_t)(b - a);
    if (!al) {
      if (hash) hash[i] = fnv_range(p, a, b);
      // long URIs: entropy over the first 255 bytes keeps u8 counts exact
      if (ent) ent[i] = entropy_range(p, a, (b - a) > 255 ? a + 255 : b, hist[threadIdx.x], clogc, lg);
      continue;
    }
    uint8_t* hh = hist[threadIdx.x];
    const int64_t ee = (b - a) > 255 ? a + 255 : b;  // entropy window
    if (ent)
      for (int k = 0; k < kBins; k += 4) *reinterpret_cast<uint32_t*>(hh + k) = 0u;
    uint64_t h = kFnvOff;
    for (int64_t w = a & ~int64_t(3); w < b; w += 4) {
      const uint32_t v = *reinterpret_cast<const uint32_t*>(p + w);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t q = w + j;
        if (q >= a && q < b) {
          const uint8_t c = lower((uint8_t)(v >> (8 * j)));
          h = (h ^ c) * kFnvPrime;
          if (ent && q < ee) {
            const int k = cbin(c);
            hh[k] = (uint8_t)(hh[k] + 1);
          }
        }
      }
    }
    if (hash) hash[i] = h;
    if (ent) ent[i] = b > a ? entropy_of_hist(hh, (int)(ee - a), clogc, lg) : 0.f;
  }
}

__global__ void k_set_probe(const uint64_t* __restrict__ h, int64_t n, const uint64_t* __restrict__ tab, uint64_t mask,
                            uint8_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = set_probe(tab, mask, h[i]);
}

}  // namespace

ONI_API int oni_domain_features(const int64_t* off, const uint8_t* chars, int64_t n, const uint64_t* top_tab,
                                uint64_t top_mask, uint64_t user_hash, int user_is_label, const float* clogc,
                                const float* lg, const uint64_t* psl_rules, uint64_t psl_rules_mask,
                                const uint64_t* psl_exc, uint64_t psl_exc_mask, int psl_max_labels,
                                uint64_t* reg_hash, uint8_t* top, int32_t* sub_len, float* sub_ent, int32_t* periods,
                                hipStream_t s) {
  if (psl_max_labels < 1 || psl_max_labels > kMaxLabels) return (int)hipErrorInvalidValue;
  DomainOut o{reg_hash, top, sub_len, sub_ent, periods, nullptr};
  const Psl psl{psl_rules, psl_rules_mask, psl_exc, psl_exc_mask, psl_max_labels};
  k_domain_features<<<oni::grid_for(n, 256, 2048), 256, 0, s>>>(off, chars, n, top_tab, top_mask, user_hash,
                                                                 user_is_label, clogc, lg, psl, o);
  return (int)hipGetLastError();
}

ONI_API int oni_string_features(const int64_t* off, const uint8_t* chars, int64_t n, const float* clogc,
                                const float* lg, uint64_t* hash, int32_t* len, float* ent, hipStream_t s) {
  k_string_features<<<oni::grid_for(n, 256, 2048), 256, 0, s>>>(off, chars, n, clogc, lg, hash, len, ent);
  return (int)hipGetLastError();
}

ONI_API int oni_set_probe(const uint64_t* h, int64_t n, const uint64_t* tab, uint64_t mask, uint8_t* out,
                          hipStream_t s) {
  k_set_probe<<<oni::grid_for(n), 256, 0, s>>>(h, n, tab, mask, out);
  return (int)hipGetLastError();
}

// ---- categorical codes by pattern table (proxy method / content type) -------------------------
// code(s) for a string s, after trimming ASCII whitespace and folding case (fold: 1 = upper,
// 2 = lower): the code of the LONGEST pattern p that matches -- exactly (mode 0) or as a prefix
// (mode 1) -- else `dflt`. The patterns of one table (≤ 32, ≤ 32 bytes each) live in LDS; one
// thread per row. The same rule as proxy.method_code / proxy.ctype_class on the host, without
// the round trip of "distinct values → host labels → table".
namespace {
constexpr int kCatMax = 32, kCatLen = 32;

__device__ __forceinline__ uint8_t fold_char(uint8_t c, int fold) {
  if (fold == 1 && c >= 'a' && c <= 'z') return (uint8_t)(c - 32);
  if (fold == 2 && c >= 'A' && c <= 'Z') return (uint8_t)(c + 32);
  return c;
}

__device__ __forceinline__ bool is_space(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' ||
                                                             c == '\v' || c == '\f'; }

__global__ __launch_bounds__(256) void k_category_codes(const int64_t* __restrict__ off,
                                                        const uint8_t* __restrict__ chars, int64_t n,
                                                        const uint8_t* __restrict__ pat, const int32_t* __restrict__ plen,
                                                        const int32_t* __restrict__ pmode,
                                                        const int32_t* __restrict__ pcode, int np, int fold, int dflt,
                                                        int32_t* __restrict__ out) {
  __shared__ uint8_t sp[kCatMax * kCatLen];
  __shared__ int32_t sl[kCatMax], sm[kCatMax], sc[kCatMax];
  for (int i = threadIdx.x; i < np * kCatLen; i += blockDim.x) sp[i] = pat[i];
  for (int i = threadIdx.x; i < np; i += blockDim.x) {
    sl[i] = plen[i];
    sm[i] = pmode[i];
    sc[i] = pcode[i];
  }
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride) {
    int64_t a = off[r], b = off[r + 1];
    while (a < b && is_space(chars[a])) ++a;
    while (b > a && is_space(chars[b - 1])) --b;
    const int64_t len = b - a;
    int best = dflt, blen = -1;
    for (int p = 0; p < np; ++p) {
      const int pl = sl[p];
      if (pl <= blen || (sm[p] == 0 ? len != pl : len < pl)) continue;
      bool ok = true;
      for (int j = 0; j < pl && ok; ++j) ok = fold_char(chars[a + j], fold) == sp[p * kCatLen + j];
      if (ok) {
        best = sc[p];
        blen = pl;
      }
    }
    out[r] = best;
  }
}
}  // namespace

ONI_API int oni_category_codes(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* pat,
                               const int32_t* plen, const int32_t* pmode, const int32_t* pcode, int np, int fold,
                               int dflt, int32_t* out, hipStream_t s) {
  if (np < 0 || np > kCatMax) return (int)hipErrorInvalidValue;
  if (n <= 0) return 0;
  k_category_codes<<<oni::grid_for(n, 256, 4096), 256, 0, s>>>(off, chars, n, pat, plen, pmode, pcode, np, fold, dflt,
                                                                out);
  return (int)hipGetLastError();
}
