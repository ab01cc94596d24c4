// K17 -- result rows → CSV text (the reference's Spark `saveAsTextFile` + `hdfs dfs -getmerge` of
// `<source>_results.csv`; oni-nfdump's CSV formatter, §2.3).
//
// The pipeline hands over the already-gathered result rows as typed columns (one value per
// output row, in output order); this formats all of them in one pass into a caller-owned buffer
// and records where every row ends, so rows from several ranks can be re-ordered by global row id
// without re-formatting. Field kinds:
//
//   0 int64 decimal          1 uint32 IPv4 dotted quad      2 unix seconds → "YYYY-MM-DD HH:MM:SS"
//   3 float64 "%g"           4 float32 "%.9g" (scores)      5 string (int64 offsets + bytes),
//   6 packed flow word (u32: dir@28 | port@11 | tbin@7 | bbin@3 | pbin, spec.flow_word_str)
//
// Strings follow Python csv.QUOTE_MINIMAL: quoted (with "" doubling) when they contain a comma,
// a quote, CR or LF. Lines end in '\n'.
#include <charconv>
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <ctime>

#include "oni_native.h"

namespace {

// matches oni355.ref.spec.PORT_111111 / PORT_333333 (port codes that render as 111111 / 333333)
constexpr uint32_t kPort111111 = 0x10000;
constexpr uint32_t kPort333333 = 0x10001;

struct Buf {
  char* p;
  int64_t cap, n = 0;
  bool overflow = false;
  void put(const char* s, size_t len) {
    if (n + (int64_t)len <= cap) std::memcpy(p + n, s, len);
    else overflow = true;
    n += (int64_t)len;
  }
  void ch(char c) {
    if (n < cap) p[n] = c;
    else overflow = true;
    ++n;
  }
};

void put_i64(Buf& b, int64_t v) {
  char t[24];
  const auto r = std::to_chars(t, t + sizeof t, v);
  b.put(t, (size_t)(r.ptr - t));
}

void put_u32(Buf& b, uint32_t v) {
  char t[12];
  const auto r = std::to_chars(t, t + sizeof t, v);
  b.put(t, (size_t)(r.ptr - t));
}

void two(char* p, int v) {
  p[0] = (char)('0' + v / 10);
  p[1] = (char)('0' + v % 10);
}

// UTC civil time without gmtime (days → y/m/d, Howard Hinnant's algorithm)
void put_time(Buf& b, int64_t unix_s) {
  int64_t days = unix_s / 86400, sec = unix_s % 86400;
  if (sec < 0) {
    sec += 86400;
    --days;
  }
  const int64_t z = days + 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  const int d = (int)(doy - (153 * mp + 2) / 5 + 1);
  const int m = (int)(mp < 10 ? mp + 3 : mp - 9);
  const int64_t y = yoe + era * 400 + (m <= 2);
  if (y < 0 || y > 9999) {  // outside 4-digit years: keep strftime's behaviour
    std::time_t t = (std::time_t)unix_s;
    std::tm tm{};
    gmtime_r(&t, &tm);
    char s[64];
    b.put(s, std::strftime(s, sizeof s, "%Y-%m-%d %H:%M:%S", &tm));
    return;
  }
  char s[19] = {0};
  s[0] = (char)('0' + y / 1000);
  s[1] = (char)('0' + (y / 100) % 10);
  s[2] = (char)('0' + (y / 10) % 10);
  s[3] = (char)('0' + y % 10);
  s[4] = '-';
  two(s + 5, m);
  s[7] = '-';
  two(s + 8, d);
  s[10] = ' ';
  two(s + 11, (int)(sec / 3600));
  s[13] = ':';
  two(s + 14, (int)(sec / 60 % 60));
  s[16] = ':';
  two(s + 17, (int)(sec % 60));
  b.put(s, 19);
}

void put_float(Buf& b, double v, int prec) {
  char t[48];
  const auto r = std::to_chars(t, t + sizeof t, v, std::chars_format::general, prec);
  b.put(t, (size_t)(r.ptr - t));
}

void put_str(Buf& b, const uint8_t* s, int64_t len) {
  bool quote = false;
  for (int64_t i = 0; i < len && !quote; ++i)
    quote = s[i] == ',' || s[i] == '"' || s[i] == '\n' || s[i] == '\r';
  if (!quote) {
    b.put(reinterpret_cast<const char*>(s), (size_t)len);
    return;
  }
  b.ch('"');
  for (int64_t i = 0; i < len; ++i) {
    if (s[i] == '"') b.ch('"');
    b.ch((char)s[i]);
  }
  b.ch('"');
}

void put_flow_word(Buf& b, uint32_t w) {
  const uint32_t d = (w >> 28) & 1, port = (w >> 11) & 0x1FFFF, tb = (w >> 7) & 0xF, bb = (w >> 3) & 0xF, pb = w & 7;
  if (d) b.put("-1_", 3);
  if (port == kPort111111) b.put("111111", 6);
  else if (port == kPort333333) b.put("333333", 6);
  else put_u32(b, port);
  b.ch('_');
  put_u32(b, tb);
  b.ch('_');
  put_u32(b, bb);
  b.ch('_');
  put_u32(b, pb);
}

}  // namespace

// Format n_rows × n_cols fields. data[c] points at the column's values (or the chars of a string
// column, whose offsets are offs[c]). Returns the byte length written (rows end at row_end[i]);
// if that exceeds cap nothing is guaranteed and the caller retries with a larger buffer.
ONI_NATIVE_API int64_t oni_csv_format(int64_t n_rows, int n_cols, const int32_t* kinds, const void* const* data,
                                      const int64_t* const* offs, char* out, int64_t cap, int64_t* row_end) {
  Buf b{out, cap};
  for (int64_t r = 0; r < n_rows; ++r) {
    for (int c = 0; c < n_cols; ++c) {
      if (c) b.ch(',');
      switch (kinds[c]) {
        case 0: put_i64(b, static_cast<const int64_t*>(data[c])[r]); break;
        case 1: {
          const uint32_t v = static_cast<const uint32_t*>(data[c])[r];
          put_u32(b, v >> 24);
          b.ch('.');
          put_u32(b, (v >> 16) & 255u);
          b.ch('.');
          put_u32(b, (v >> 8) & 255u);
          b.ch('.');
          put_u32(b, v & 255u);
          break;
        }
        case 2: put_time(b, static_cast<const int64_t*>(data[c])[r]); break;
        case 3: put_float(b, static_cast<const double*>(data[c])[r], 6); break;
        case 4: put_float(b, (double)static_cast<const float*>(data[c])[r], 9); break;
        case 5: {
          const int64_t* o = offs[c];
          put_str(b, static_cast<const uint8_t*>(data[c]) + o[r], o[r + 1] - o[r]);
          break;
        }
        case 6: put_flow_word(b, static_cast<const uint32_t*>(data[c])[r]); break;
        default: return -1;
      }
    }
    b.ch('\n');
    row_end[r] = b.n;
  }
  return b.n;
}
