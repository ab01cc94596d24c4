// oni-fuzz: drive the C++ decoders on arbitrary bytes (used by tests/test_sanitize.py with the
// ASan/UBSan build flavour: `python tools/build.py --only native --sanitize` → oni-fuzz_asan).
//   oni-fuzz <csv|proxy|pcap|nfcapd|lzo|lz4> <file>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "oni_native.h"

extern "C" {
int64_t oni_csv_count_rows(const char* path, int skip_header, int threads);
int64_t oni_csv_parse(const char* path, int skip_header, int n_fields, const int* kinds, void** outs, int64_t cap_rows,
                      uint8_t* valid, char sep, int threads);
void* oni_pcap_dns_open(const char* path, int threads);
int oni_pcap_dns_sizes(void* h, int64_t* rows, int64_t* nb, int64_t* ab, int64_t* pk);
int oni_pcap_dns_fetch(void* h, int64_t* ts, int32_t* fl, uint32_t* s, uint32_t* d, int32_t* qt, int32_t* qc,
                       int32_t* rc, int64_t* noff, uint8_t* names, int64_t* aoff, uint8_t* as);
void oni_pcap_dns_free(void* h);
void* oni_nfcapd_open(const char* path);
int oni_nfcapd_info(void* h, int64_t* n, int64_t* blocks, int64_t* skipped, char* err, int err_len);
int oni_nfcapd_fetch(void* h, int64_t* a64, int32_t* a32, uint32_t* rip);
void oni_nfcapd_free(void* h);
int oni_lzo1x_decompress(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap, int64_t* out_len);
int oni_lz4_decompress(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap, int64_t* out_len);
}

static std::vector<uint8_t> slurp(const char* p) {
  std::vector<uint8_t> b;
  FILE* f = std::fopen(p, "rb");
  if (!f) return b;
  uint8_t buf[65536];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
  std::fclose(f);
  return b;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: oni-fuzz <csv|proxy|pcap|nfcapd|lzo|lz4> <file>\n");
    return 2;
  }
  const char* mode = argv[1];
  const char* path = argv[2];
  if (!std::strcmp(mode, "csv") || !std::strcmp(mode, "proxy")) {
    const bool proxy = !std::strcmp(mode, "proxy");
    const int64_t n = oni_csv_count_rows(path, 1, 2);
    if (n < 0) return 0;
    const int nf = 8;
    int kinds[nf] = {6, 1, 2, 3, 4, 5, 7, 1};  // TIME I64 F64 IPV4 PROTO FLAGS STR I64
    std::vector<int64_t> t(n + 1), i64(n + 1), s(2 * n + 2), last(n + 1);
    std::vector<double> f(n + 1);
    std::vector<uint32_t> ip(n + 1);
    std::vector<int32_t> pr(n + 1), fl(n + 1);
    void* outs[nf] = {t.data(), i64.data(), f.data(), ip.data(), pr.data(), fl.data(), s.data(), last.data()};
    std::vector<uint8_t> valid(n + 1);
    oni_csv_parse(path, 1, nf, kinds, outs, n, valid.data(), proxy ? ' ' : ',', 2);
    return 0;
  }
  if (!std::strcmp(mode, "pcap")) {
    void* h = oni_pcap_dns_open(path, 2);
    int64_t rows, nb, ab, pk;
    if (oni_pcap_dns_sizes(h, &rows, &nb, &ab, &pk) == 0) {
      std::vector<int64_t> ts(rows + 1), noff(rows + 2), aoff(rows + 2);
      std::vector<int32_t> fl(rows + 1), qt(rows + 1), qc(rows + 1), rc(rows + 1);
      std::vector<uint32_t> sa(rows + 1), da(rows + 1);
      std::vector<uint8_t> names(nb + 1), as(ab + 1);
      oni_pcap_dns_fetch(h, ts.data(), fl.data(), sa.data(), da.data(), qt.data(), qc.data(), rc.data(), noff.data(),
                         names.data(), aoff.data(), as.data());
    }
    oni_pcap_dns_free(h);
    return 0;
  }
  if (!std::strcmp(mode, "nfcapd")) {
    void* h = oni_nfcapd_open(path);
    int64_t n, blocks, skipped;
    char err[256];
    oni_nfcapd_info(h, &n, &blocks, &skipped, err, sizeof err);
    std::vector<int64_t> a64(8 * (n + 1));
    std::vector<int32_t> a32(14 * (n + 1));
    std::vector<uint32_t> rip(n + 1);
    oni_nfcapd_fetch(h, a64.data(), a32.data(), rip.data());
    oni_nfcapd_free(h);
    return 0;
  }
  const auto b = slurp(path);
  std::vector<uint8_t> out(1 << 20);
  int64_t n = 0;
  if (!std::strcmp(mode, "lzo")) oni_lzo1x_decompress(b.data(), (int64_t)b.size(), out.data(), (int64_t)out.size(), &n);
  if (!std::strcmp(mode, "lz4")) oni_lz4_decompress(b.data(), (int64_t)b.size(), out.data(), (int64_t)out.size(), &n);
  return 0;
}
