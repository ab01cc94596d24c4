// IPv4 / IPv6 address text <-> binary for the flow decoders (C01 / nfdump CSV) and the result
// formatter. IPv6 flows keep their 16-byte addresses; the pipeline gives every distinct IPv6
// address of a day an exact 32-bit document key (oni355/pipeline/flow.py ipv6_doc_keys).
#include <arpa/inet.h>

#include <cstring>

#include "oni_native.h"

// spans[n][2] (begin, end) into buf: dotted IPv4 -> v4[i] (is_v6[i] = 0); IPv6 text ->
// v6[i][16] (is_v6[i] = 1, v4[i] = 0); anything else -> is_v6[i] = 2 (unparsable).
ONI_NATIVE_API int64_t oni_ip_parse_spans(const uint8_t* buf, const int64_t* spans, int64_t n, uint32_t* v4,
                                          uint8_t* v6, uint8_t* is_v6) {
  int64_t bad = 0;
  char tmp[64];
  for (int64_t i = 0; i < n; ++i) {
    const int64_t b = spans[2 * i], e = spans[2 * i + 1];
    const int64_t len = e - b;
    v4[i] = 0;
    std::memset(v6 + 16 * i, 0, 16);
    if (len <= 0 || len >= (int64_t)sizeof tmp) {
      is_v6[i] = 2;
      ++bad;
      continue;
    }
    std::memcpy(tmp, buf + b, (size_t)len);
    tmp[len] = 0;
    in_addr a4;
    if (inet_pton(AF_INET, tmp, &a4) == 1) {
      v4[i] = ntohl(a4.s_addr);
      is_v6[i] = 0;
    } else if (inet_pton(AF_INET6, tmp, v6 + 16 * i) == 1) {
      is_v6[i] = 1;
    } else {
      is_v6[i] = 2;
      ++bad;
    }
  }
  return bad;
}

// RFC 5952 text of the 16-byte addresses addrs[i * stride ...] of the rows with is_v6[i] = 1
// (empty for the others). Two-phase: buf == nullptr only fills off[n + 1] (running byte offsets).
ONI_NATIVE_API int oni_ipv6_text(const uint8_t* addrs, int64_t stride, const uint8_t* is_v6, int64_t n, int64_t* off,
                                 char* buf) {
  off[0] = 0;
  char t[INET6_ADDRSTRLEN];
  for (int64_t i = 0; i < n; ++i) {
    size_t l = 0;
    if (is_v6[i] == 1) {
      if (!inet_ntop(AF_INET6, addrs + i * stride, t, sizeof t)) return 1;
      l = std::strlen(t);
      if (buf) std::memcpy(buf + off[i], t, l);
    }
    off[i + 1] = off[i] + (int64_t)l;
  }
  return 0;
}

// IPv6 text -> 16 bytes (1 on success)
ONI_NATIVE_API int oni_ipv6_parse(const char* s, uint8_t* out16) { return inet_pton(AF_INET6, s, out16) == 1; }
