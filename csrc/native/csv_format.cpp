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
//   7 packed u64 word rendered as '_'-joined decimal fields (DNS / proxy word_str); offs[c] holds
//     the field spec [n_fields, shift_0, mask_0, shift_1, mask_1, ...]
//   8 string, or -- where it is empty -- unix seconds as kind 2 (DNS frame_time of synthetic /
//     columnar rows); data[c] → StrCol {chars, offsets, rows, unix seconds (per output row)}
//   9 string read straight from a whole column: data[c] → StrCol {chars, offsets, rows}; output
//     row r is column row rows[r] (no host-side gather of the selected strings)
//
// Strings follow Python csv.QUOTE_MINIMAL: quoted (with "" doubling) when they contain a comma,
// a quote, CR or LF. Lines end in '\n'.
#include <charconv>
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <atomic>
#include <thread>
#include <vector>

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

void put_packed(Buf& b, uint64_t w, const int64_t* spec) {
  const int64_t nf = spec[0];
  for (int64_t f = 0; f < nf; ++f) {
    if (f) b.ch('_');
    char t[24];
    const uint64_t v = (w >> spec[1 + 2 * f]) & (uint64_t)spec[2 + 2 * f];
    const auto r = std::to_chars(t, t + sizeof t, v);
    b.put(t, (size_t)(r.ptr - t));
  }
}

struct StrCol {
  const uint8_t* chars;
  const int64_t* offs;
  const int64_t* rows;  // nullable: identity
  const int64_t* unix_s;
};

// Rows [r0, r1) into b; row_end[r] is relative to b's start. Returns false on an unknown kind.
// The string columns are read at random rows of day-sized columns: each field is a cache miss, so
// the offsets of row r + 2·kAhead and the characters of row r + kAhead are prefetched.
constexpr int64_t kAhead = 8;

void prefetch_row(int n_cols, const int32_t* kinds, const void* const* data, int64_t r, bool chars) {
  for (int c = 0; c < n_cols; ++c) {
    if (kinds[c] != 8 && kinds[c] != 9) continue;
    const auto* st = static_cast<const StrCol*>(data[c]);
    const int64_t i = st->rows ? st->rows[r] : r;
    if (chars) __builtin_prefetch(st->chars + st->offs[i]);
    else __builtin_prefetch(st->offs + i);
  }
}

bool format_rows(int64_t r0, int64_t r1, int n_cols, const int32_t* kinds, const void* const* data,
                 const int64_t* const* offs, Buf& b, int64_t* row_end) {
  for (int64_t r = r0; r < r1; ++r) {
    if (r + 2 * kAhead < r1) prefetch_row(n_cols, kinds, data, r + 2 * kAhead, false);
    if (r + kAhead < r1) prefetch_row(n_cols, kinds, data, r + kAhead, true);
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
        case 7: put_packed(b, static_cast<const uint64_t*>(data[c])[r], offs[c]); break;
        case 8:
        case 9: {
          const auto* st = static_cast<const StrCol*>(data[c]);
          const int64_t i = st->rows ? st->rows[r] : r;
          const int64_t len = st->offs[i + 1] - st->offs[i];
          if (len || kinds[c] == 9) put_str(b, st->chars + st->offs[i], len);
          else put_time(b, st->unix_s[r]);
          break;
        }
        default: return false;
      }
    }
    b.ch('\n');
    row_end[r] = b.n;
  }
  return true;
}

}  // namespace

// Format n_rows × n_cols fields. data[c] points at the column's values (or the chars of a string
// column, whose offsets are offs[c]). Returns the byte length written (rows end at row_end[i]);
// if that exceeds cap nothing is guaranteed and the caller retries with a larger buffer; -1 on an
// unknown kind. Large row counts are formatted in parallel row blocks (private buffers, then one
// copy into `out`), which also overlaps the cache misses of the random-row string reads.
ONI_NATIVE_API int64_t oni_csv_format(int64_t n_rows, int n_cols, const int32_t* kinds, const void* const* data,
                                      const int64_t* const* offs, char* out, int64_t cap, int64_t* row_end) {
  const int64_t kBlockRows = 512;  // ≥ 2 blocks before threads start (thread start ≈ tens of µs)
  const int64_t nb = (n_rows + kBlockRows - 1) / kBlockRows;
  if (nb <= 1) {
    Buf b{out, cap};
    if (!format_rows(0, n_rows, n_cols, kinds, data, offs, b, row_end)) return -1;
    return b.n;
  }
  std::vector<std::vector<char>> parts((size_t)nb);
  std::vector<int64_t> len((size_t)nb, 0);
  std::atomic<int> bad{0};
  std::atomic<int64_t> next{0};
  auto work = [&] {
    for (int64_t k = next.fetch_add(1); k < nb; k = next.fetch_add(1)) {
      const int64_t r0 = k * kBlockRows, r1 = std::min(n_rows, r0 + kBlockRows);
      std::vector<char>& v = parts[(size_t)k];
      v.resize((size_t)std::max<int64_t>(4096, cap / nb + 4096));
      for (;;) {
        Buf b{v.data(), (int64_t)v.size()};
        if (!format_rows(r0, r1, n_cols, kinds, data, offs, b, row_end)) {
          bad = 1;
          break;
        }
        if (!b.overflow) {
          len[(size_t)k] = b.n;
          break;
        }
        v.resize((size_t)b.n);
      }
    }
  };
  const int nt = (int)std::min<int64_t>(nb, std::max(1u, std::min(8u, std::thread::hardware_concurrency())));
  std::vector<std::thread> ts;
  for (int t = 1; t < nt; ++t) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
  if (bad) return -1;
  int64_t total = 0;
  for (int64_t k = 0; k < nb; ++k) total += len[(size_t)k];
  if (total > cap) return total;
  int64_t base = 0;
  for (int64_t k = 0; k < nb; ++k) {
    const int64_t r0 = k * kBlockRows, r1 = std::min(n_rows, r0 + kBlockRows);
    std::memcpy(out + base, parts[(size_t)k].data(), (size_t)len[(size_t)k]);
    for (int64_t r = r0; r < r1; ++r) row_end[r] += base;
    base += len[(size_t)k];
  }
  return total;
}
