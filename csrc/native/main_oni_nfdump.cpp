// oni-nfdump -- nfcapd → ONI flow CSV (the oni-nfdump fork's `nfdump -r <file> -o csv` role in the
// reference ingest pipeline, SURVEY.md §2.2 C01 / §2.3 "oni-nfdump (nfdump binary: nfcapd decode +
// CSV formatter)"; reference submodule `oni-nfdump` at /root/reference/.gitmodules:13-15 is an
// empty gitlink, so the output format is ONI's 27-field flow schema).
//
//   oni-nfdump -r nfcapd.201607080000 [-r more ...] [-o oni|nfdump] [-q] [-w out.csv]
//
// -o oni    (default) header + rows in the Hive flow-table order oni355.io.decoders reads back:
//           treceived,tryear,trmonth,trday,trhour,trminute,trsec,tdur,sip,dip,sport,dport,proto,
//           flag,fwd,stos,ipkt,ibyt,opkt,obyt,input,output,sas,das,dtos,dir,rip
// -o nfdump stock `nfdump -o csv` header names (ts,te,td,sa,da,sp,dp,pr,flg,...)
// -q        no header
//
// Decoding is the library's (csrc/io/nfcapd.cpp: LAYOUT_VERSION_1, uncompressed / LZO1X / LZ4 /
// bzip2 blocks, extension maps); formatting is a single pass into a 1 MiB output buffer.
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <arpa/inet.h>

#include <ctime>
#include <string>
#include <vector>

#include "oni_native.h"

extern "C" {
void* oni_nfcapd_open(const char* path);
int oni_nfcapd_info(void* hp, int64_t* n_flows, int64_t* blocks, int64_t* skipped, char* err, int err_len);
int oni_nfcapd_fetch(void* hp, int64_t* out_i64, int32_t* out_i32, uint32_t* out_rip);
int oni_nfcapd_fetch_v6(void* hp, uint8_t* is_v6, uint8_t* addrs);
void oni_nfcapd_free(void* hp);
}

namespace {

struct Out {
  FILE* f;
  std::vector<char> buf;
  size_t n = 0;
  explicit Out(FILE* fp) : f(fp), buf(1 << 20) {}
  ~Out() { flush(); }
  void flush() {
    if (n) std::fwrite(buf.data(), 1, n, f);
    n = 0;
  }
  void put(const char* s, size_t len) {
    if (n + len > buf.size()) flush();
    std::memcpy(buf.data() + n, s, len);
    n += len;
  }
  void str(const char* s) { put(s, std::strlen(s)); }
  void i64(int64_t v) {
    char t[24];
    put(t, (size_t)std::snprintf(t, sizeof t, "%" PRId64, v));
  }
  void ip(uint32_t v) {
    char t[16];
    put(t, (size_t)std::snprintf(t, sizeof t, "%u.%u.%u.%u", v >> 24, (v >> 16) & 255u, (v >> 8) & 255u, v & 255u));
  }
  void time(int64_t unix_s) {
    std::time_t t = (std::time_t)unix_s;
    std::tm tm{};
    gmtime_r(&t, &tm);
    char s[32];
    put(s, std::strftime(s, sizeof s, "%Y-%m-%d %H:%M:%S", &tm));
  }
  void c() { put(",", 1); }
  void nl() { put("\n", 1); }
};

const char* proto_name(int p) {
  switch (p) {
    case 1: return "ICMP";
    case 6: return "TCP";
    case 17: return "UDP";
    case 47: return "GRE";
    case 50: return "ESP";
    case 58: return "ICMP6";
    default: return nullptr;
  }
}

void flags_str(int f, char* s) {  // nfdump order U A P R S F, '.' when unset
  const char* sym = "UAPRSF";
  const int bit[6] = {32, 16, 8, 4, 2, 1};
  for (int i = 0; i < 6; ++i) s[i] = (f & bit[i]) ? sym[i] : '.';
  s[6] = 0;
}

int usage() {
  std::fprintf(stderr, "usage: oni-nfdump -r <nfcapd file> [-r ...] [-o oni|nfdump] [-q] [-w out.csv]\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<std::string> files;
  std::string fmt = "oni", out_path;
  bool header = true;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "-r" && i + 1 < argc) files.push_back(argv[++i]);
    else if (a == "-o" && i + 1 < argc) fmt = argv[++i];
    else if (a == "-w" && i + 1 < argc) out_path = argv[++i];
    else if (a == "-q") header = false;
    else return usage();
  }
  if (files.empty() || (fmt != "oni" && fmt != "nfdump")) return usage();
  FILE* fp = out_path.empty() ? stdout : std::fopen(out_path.c_str(), "w");
  if (!fp) {
    std::fprintf(stderr, "oni-nfdump: cannot write %s\n", out_path.c_str());
    return 1;
  }
  int rc = 0;
  {
    Out o(fp);
    if (header) {
      o.str(fmt == "oni" ? "treceived,tryear,trmonth,trday,trhour,trminute,trsec,tdur,sip,dip,sport,dport,proto,flag,"
                           "fwd,stos,ipkt,ibyt,opkt,obyt,input,output,sas,das,dtos,dir,rip\n"
                         : "ts,te,td,sa,da,sp,dp,pr,flg,fwd,stos,ipkt,ibyt,opkt,obyt,in,out,sas,das,dtos,dir,ra\n");
    }
    for (const auto& path : files) {
      void* h = oni_nfcapd_open(path.c_str());
      int64_t n = 0, blocks = 0, skipped = 0;
      char err[256];
      if (oni_nfcapd_info(h, &n, &blocks, &skipped, err, sizeof err) != 0) {
        std::fprintf(stderr, "oni-nfdump: %s: %s\n", path.c_str(), err);
        oni_nfcapd_free(h);
        rc = 1;
        continue;
      }
      std::vector<int64_t> a64((size_t)n * 8);
      std::vector<int32_t> a32((size_t)n * 14);
      std::vector<uint32_t> rip((size_t)n);
      std::vector<uint8_t> v6((size_t)n), a6((size_t)n * 32);
      oni_nfcapd_fetch(h, a64.data(), a32.data(), rip.data());
      oni_nfcapd_fetch_v6(h, v6.data(), a6.data());
      oni_nfcapd_free(h);
      char fl[8], td[32];
      for (int64_t i = 0; i < n; ++i) {
        const int64_t* x = &a64[(size_t)i * 8];
        const int32_t* y = &a32[(size_t)i * 14];
        const int64_t first_s = x[0] / 1000;
        std::snprintf(td, sizeof td, "%.3f", (double)(x[1] - x[0]) / 1000.0);
        const char* pn = proto_name(y[2]);
        flags_str(y[3], fl);
        if (fmt == "oni") {
          std::time_t t = (std::time_t)first_s;
          std::tm tm{};
          gmtime_r(&t, &tm);
          o.time(first_s); o.c();
          o.i64(tm.tm_year + 1900); o.c(); o.i64(tm.tm_mon + 1); o.c(); o.i64(tm.tm_mday); o.c();
          o.i64(tm.tm_hour); o.c(); o.i64(tm.tm_min); o.c(); o.i64(tm.tm_sec); o.c();
          o.str(td); o.c();
        } else {
          o.time(first_s); o.c(); o.time(x[1] / 1000); o.c(); o.str(td); o.c();
        }
        if (v6[(size_t)i]) {  // IPv6 flow: RFC 5952 text of both addresses
          char a[INET6_ADDRSTRLEN], b[INET6_ADDRSTRLEN];
          inet_ntop(AF_INET6, &a6[(size_t)i * 32], a, sizeof a);
          inet_ntop(AF_INET6, &a6[(size_t)i * 32 + 16], b, sizeof b);
          o.str(a); o.c(); o.str(b); o.c();
        } else {
          o.ip((uint32_t)y[12]); o.c(); o.ip((uint32_t)y[13]); o.c();
        }
        o.i64(y[0]); o.c(); o.i64(y[1]); o.c();
        if (pn) o.str(pn); else o.i64(y[2]);
        o.c(); o.str(fl); o.c();
        o.i64(y[4]); o.c(); o.i64(y[5]); o.c();                    // fwd, stos
        o.i64(x[3]); o.c(); o.i64(x[4]); o.c(); o.i64(x[5]); o.c(); o.i64(x[6]); o.c();  // ipkt ibyt opkt obyt
        o.i64(y[8]); o.c(); o.i64(y[9]); o.c(); o.i64(y[10]); o.c(); o.i64(y[11]); o.c();  // in out sas das
        o.i64(y[6]); o.c(); o.i64(y[7]); o.c();                    // dtos, dir
        o.ip(rip[(size_t)i]); o.nl();
      }
      if (skipped) std::fprintf(stderr, "oni-nfdump: %s: %" PRId64 " records skipped\n", path.c_str(), skipped);
    }
  }
  if (fp != stdout) std::fclose(fp);
  return rc;
}
