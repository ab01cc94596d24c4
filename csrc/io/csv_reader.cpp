// Multithreaded typed CSV decoder (nfdump / oni-nfdump CSV, tshark field CSV, generic).
//
// Replaces the reference's `nfdump -o csv` → `hadoop fs -put` → Hive CSV staging table path
// (oni-ingest flow worker, SURVEY.md §2.2 C01/C06, [U-M]): the file is memory-mapped, split into
// per-thread byte ranges at line boundaries, lines are counted in parallel, and every thread parses
// its range straight into column arrays (no intermediate strings). The field → column mapping is
// header-driven (computed in Python, oni355/io/decoders.py), so both ONI's 27-field CSV and stock
// nfdump CSV decode through the same code.
#include <fcntl.h>
#include <omp.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <ctime>
#include <vector>

#include "../native/oni_native.h"

namespace {

enum Kind : int { SKIP = 0, I64 = 1, F64 = 2, IPV4 = 3, PROTO = 4, FLAGS = 5, TIME = 6, STR = 7 };

struct Mapped {
  const char* p = nullptr;
  size_t n = 0;
  int fd = -1;
  bool open(const char* path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0) return false;
    n = (size_t)st.st_size;
    if (n == 0) return true;
    void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) return false;
    madvise(m, n, MADV_SEQUENTIAL);
    p = (const char*)m;
    return true;
  }
  ~Mapped() {
    if (p) munmap((void*)p, n);
    if (fd >= 0) ::close(fd);
  }
};

// byte ranges [b[i], b[i+1]) each starting at a line start
std::vector<size_t> split(const Mapped& m, int parts, size_t start) {
  std::vector<size_t> b(parts + 1, m.n);
  b[0] = start;
  for (int i = 1; i < parts; ++i) {
    size_t pos = start + (m.n - start) * (size_t)i / parts;
    while (pos < m.n && m.p[pos - 1] != '\n') ++pos;
    b[i] = pos < b[i - 1] ? b[i - 1] : pos;
  }
  return b;
}

size_t header_end(const Mapped& m, int skip_header) {
  if (!skip_header) return 0;
  const void* nl = m.n ? std::memchr(m.p, '\n', m.n) : nullptr;
  return nl ? (size_t)((const char*)nl - m.p) + 1 : m.n;
}

int64_t count_lines(const char* p, size_t lo, size_t hi) {
  int64_t c = 0;
  size_t i = lo;
  while (i < hi) {
    const void* nl = std::memchr(p + i, '\n', hi - i);
    if (!nl) {
      bool blank = true;
      for (size_t j = i; j < hi; ++j)
        if (p[j] != '\r' && p[j] != ' ') blank = false;
      if (!blank) ++c;
      break;
    }
    const size_t e = (size_t)((const char*)nl - p);
    if (e > i && !(e == i + 1 && p[i] == '\r')) ++c;
    i = e + 1;
  }
  return c;
}

inline bool parse_i64(const char* s, const char* e, int64_t* out) {
  while (s < e && (*s == ' ' || *s == '"')) ++s;
  while (e > s && (e[-1] == ' ' || e[-1] == '"' || e[-1] == '\r')) --e;
  if (s == e) {
    *out = 0;
    return true;
  }
  bool neg = false;
  if (*s == '-') {
    neg = true;
    ++s;
  }
  int64_t v = 0;
  const char* dot = nullptr;
  for (const char* q = s; q < e; ++q) {
    if (*q == '.') {
      dot = q;
      break;
    }
    if (*q < '0' || *q > '9') {
      // nfdump scales large counters: "1.2 M" / "3 G"
      char* endp;
      double d = std::strtod(s, &endp);
      while (endp < e && *endp == ' ') ++endp;
      if (endp < e && (*endp == 'M' || *endp == 'G' || *endp == 'K')) {
        d *= *endp == 'M' ? 1e6 : (*endp == 'G' ? 1e9 : 1e3);
        *out = (int64_t)(neg ? -d : d);
        return true;
      }
      return false;
    }
    v = v * 10 + (*q - '0');
  }
  if (dot) {
    char* endp;
    double d = std::strtod(s, &endp);
    while (endp < e && *endp == ' ') ++endp;
    if (endp < e && (*endp == 'M' || *endp == 'G' || *endp == 'K')) d *= *endp == 'M' ? 1e6 : (*endp == 'G' ? 1e9 : 1e3);
    v = (int64_t)d;
  }
  *out = neg ? -v : v;
  return true;
}

inline bool parse_f64(const char* s, const char* e, double* out) {
  while (s < e && (*s == ' ' || *s == '"')) ++s;
  if (s == e) {
    *out = 0;
    return true;
  }
  char buf[64];
  size_t n = (size_t)(e - s) < sizeof(buf) - 1 ? (size_t)(e - s) : sizeof(buf) - 1;
  std::memcpy(buf, s, n);
  buf[n] = 0;
  char* endp;
  *out = std::strtod(buf, &endp);
  return endp != buf;
}

inline bool parse_ip(const char* s, const char* e, uint32_t* out) {
  while (s < e && (*s == ' ' || *s == '"')) ++s;
  uint32_t ip = 0;
  int parts = 0;
  uint32_t cur = 0;
  bool any = false;
  for (const char* q = s; q < e && *q != ' ' && *q != '"' && *q != '\r'; ++q) {
    if (*q == '.') {
      if (!any || cur > 255) return false;
      ip = (ip << 8) | cur;
      cur = 0;
      any = false;
      ++parts;
    } else if (*q >= '0' && *q <= '9') {
      cur = cur * 10 + (*q - '0');
      any = true;
    } else {
      // IPv6 or garbage: fold to a 32-bit FNV-1a hash (documents are keyed by u32)
      uint32_t h = 2166136261u;
      for (const char* r = s; r < e && *r != '"' && *r != '\r'; ++r) h = (h ^ (uint8_t)*r) * 16777619u;
      *out = h;
      return true;
    }
  }
  if (parts != 3 || !any || cur > 255) return false;
  *out = (ip << 8) | cur;
  return true;
}

inline int32_t parse_proto(const char* s, const char* e) {
  while (s < e && (*s == ' ' || *s == '"')) ++s;
  while (e > s && (e[-1] == ' ' || e[-1] == '"' || e[-1] == '\r')) --e;
  const size_t n = (size_t)(e - s);
  if (n == 3 && !strncasecmp(s, "TCP", 3)) return 6;
  if (n == 3 && !strncasecmp(s, "UDP", 3)) return 17;
  if (n == 4 && !strncasecmp(s, "ICMP", 4)) return 1;
  if (n == 3 && !strncasecmp(s, "GRE", 3)) return 47;
  if (n == 3 && !strncasecmp(s, "ESP", 3)) return 50;
  if (n == 6 && !strncasecmp(s, "ICMP6", 5)) return 58;
  int64_t v = 0;
  return parse_i64(s, e, &v) ? (int32_t)v : -1;
}

// nfdump flag string ".AP.SF" (order U A P R S F; also "CE" prefixes) -> bit mask; numeric passthrough
inline int32_t parse_flags(const char* s, const char* e) {
  while (s < e && (*s == ' ' || *s == '"')) ++s;
  if (s < e && *s >= '0' && *s <= '9') {
    int64_t v = 0;
    parse_i64(s, e, &v);
    return (int32_t)v;
  }
  int32_t f = 0;
  for (const char* q = s; q < e; ++q) switch (*q) {
      case 'F': f |= 1; break;
      case 'S': f |= 2; break;
      case 'R': f |= 4; break;
      case 'P': f |= 8; break;
      case 'A': f |= 16; break;
      case 'U': f |= 32; break;
      case 'E': f |= 64; break;
      case 'C': f |= 128; break;
      default: break;
    }
  return f;
}

// "YYYY-MM-DD HH:MM:SS[.mmm]" (UTC) or epoch seconds -> unix seconds
inline bool parse_time(const char* s, const char* e, int64_t* out) {
  while (s < e && (*s == ' ' || *s == '"')) ++s;
  if (e - s >= 19 && s[4] == '-' && s[7] == '-') {
    struct tm t;
    std::memset(&t, 0, sizeof t);
    auto num = [](const char* p, int n) {
      int v = 0;
      for (int i = 0; i < n; ++i) v = v * 10 + (p[i] - '0');
      return v;
    };
    t.tm_year = num(s, 4) - 1900;
    t.tm_mon = num(s + 5, 2) - 1;
    t.tm_mday = num(s + 8, 2);
    t.tm_hour = num(s + 11, 2);
    t.tm_min = num(s + 14, 2);
    t.tm_sec = num(s + 17, 2);
    *out = (int64_t)timegm(&t);
    return true;
  }
  double d;
  if (!parse_f64(s, e, &d)) return false;
  *out = (int64_t)d;
  return true;
}

}  // namespace

ONI_NATIVE_API int64_t oni_csv_count_rows(const char* path, int skip_header, int threads) {
  Mapped m;
  if (!m.open(path)) return -1;
  if (m.n == 0) return 0;
  const size_t h = header_end(m, skip_header);
  const int T = threads > 0 ? threads : omp_get_max_threads();
  auto b = split(m, T, h);
  int64_t total = 0;
#pragma omp parallel for num_threads(T) reduction(+ : total)
  for (int i = 0; i < T; ++i) total += count_lines(m.p, b[i], b[i + 1]);
  return total;
}

// kinds[f] per CSV field; outs[f] = destination array (nullptr to skip). STR fields write
// (begin, end) byte offsets into outs[f] as int64 pairs so Python can slice the mapped bytes.
// valid[row] = 1 when the row parsed. Returns rows seen, or <0 on error.
ONI_NATIVE_API int64_t oni_csv_parse(const char* path, int skip_header, int n_fields, const int* kinds, void** outs,
                                     int64_t cap_rows, uint8_t* valid, char sep, int threads) {
  Mapped m;
  if (!m.open(path)) return -1;
  if (m.n == 0) return 0;
  const size_t h = header_end(m, skip_header);
  const int T = threads > 0 ? threads : omp_get_max_threads();
  auto b = split(m, T, h);
  std::vector<int64_t> start(T + 1, 0);
  for (int i = 0; i < T; ++i) start[i + 1] = start[i] + count_lines(m.p, b[i], b[i + 1]);
  if (start[T] > cap_rows) return -2;
#pragma omp parallel for num_threads(T) schedule(static, 1)
  for (int t = 0; t < T; ++t) {
    int64_t row = start[t];
    size_t i = b[t];
    const size_t hi = b[t + 1];
    std::vector<const char*> fs(n_fields + 1), fe(n_fields + 1);
    while (i < hi) {
      const void* nl = std::memchr(m.p + i, '\n', hi - i);
      size_t e = nl ? (size_t)((const char*)nl - m.p) : hi;
      size_t le = e;
      if (le > i && m.p[le - 1] == '\r') --le;
      if (le == i) {
        i = e + 1;
        continue;
      }
      // tokenize (quotes respected)
      int nf = 0;
      size_t fsb = i;
      bool inq = false;
      for (size_t q = i; q <= le; ++q) {
        if (q < le && m.p[q] == '"') inq = !inq;
        if (q == le || (m.p[q] == sep && !inq)) {
          if (nf < n_fields) {
            fs[nf] = m.p + fsb;
            fe[nf] = m.p + q;
          }
          ++nf;
          fsb = q + 1;
        }
      }
      bool ok = nf >= n_fields;
      for (int f = 0; ok && f < n_fields; ++f) {
        void* o = outs[f];
        if (!o || kinds[f] == SKIP) continue;
        switch (kinds[f]) {
          case I64: ok = parse_i64(fs[f], fe[f], (int64_t*)o + row); break;
          case F64: ok = parse_f64(fs[f], fe[f], (double*)o + row); break;
          case IPV4: ok = parse_ip(fs[f], fe[f], (uint32_t*)o + row); break;
          case PROTO: ((int32_t*)o)[row] = parse_proto(fs[f], fe[f]); break;
          case FLAGS: ((int32_t*)o)[row] = parse_flags(fs[f], fe[f]); break;
          case TIME: ok = parse_time(fs[f], fe[f], (int64_t*)o + row); break;
          case STR: {
            const char* s = fs[f];
            const char* se = fe[f];
            if (se > s && *s == '"') {
              ++s;
              if (se > s && se[-1] == '"') --se;
            }
            ((int64_t*)o)[2 * row] = (int64_t)(s - m.p);
            ((int64_t*)o)[2 * row + 1] = (int64_t)(se - m.p);
            break;
          }
          default: break;
        }
      }
      valid[row] = ok ? 1 : 0;
      ++row;
      i = e + 1;
    }
  }
  return start[T];
}
