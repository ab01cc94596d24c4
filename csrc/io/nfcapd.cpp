// nfcapd binary reader/writer -- the oni-nfdump decode path ([U-M] layout).
//
// The reference ran a fork of nfdump 1.6.x (`nfdump -r nfcapd.YYYYMMDDhhmm -o csv`) inside every
// flow ingest worker. This is an independent reader for nfdump's LAYOUT_VERSION_1 files written
// from the publicly documented structure, emitting flow-schema columns directly:
//
//   file_header (magic 0xA50C, version 1, flags, NumBlocks, ident[128])   140 B
//   stat_record                                                            144 B + 16 B
//   NumBlocks × { data_block_header {NumRecords, size, id = 2, flags}  12 B, records... }
//   record: {u16 type, u16 size, ...}; type 2 = extension map, type 10 = common record
//   common record: flags, ext_map, msec_first/last, first/last, fwd_status, tcp_flags, prot, tos,
//                  srcport, dstport, exporter_sysid, biFlowDir, flowEndReason  (32 B) then
//                  src/dst address (v4 or v6), packets (4/8 B), bytes (4/8 B), map extensions.
//   block compression: none, LZO1X (own decompressor), LZ4 block (own decompressor), bzip2
//   (the system libbz2, resolved with dlopen: the image ships the library but not its header).
//
// Not verifiable against the reference's submodule (empty gitlink): the format
// is pinned by tests against our own writer (oni_nfcapd_write) and hand-built LZO/LZ4 streams.
#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../native/oni_native.h"

namespace {

constexpr uint16_t kMagic = 0xA50C;
constexpr uint32_t kFlagLZO = 0x1, kFlagBZ2 = 0x8, kFlagLZ4 = 0x10;

// extension id -> payload size (bytes); 0 = unknown (stop decoding the record's extensions)
int ext_size(int id) {
  static const int sz[] = {0, 0, 0, 0, 4, 8, 4, 8, 4, 4, 16, 4, 16, 4, 4, 8, 4, 8, 4, 8, 16, 16, 40, 4, 16, 4, 8, 8};
  return (id >= 0 && id < (int)(sizeof(sz) / sizeof(sz[0]))) ? sz[id] : 0;
}

// ---- bzip2 (system libbz2.so.1, BZ2_bzBuffToBuff* one-shot API) --------------------------------
using BzDecFn = int (*)(char*, unsigned*, char*, unsigned, int, int);
using BzEncFn = int (*)(char*, unsigned*, char*, unsigned, int, int, int);
constexpr int kBzOk = 0, kBzOutbuffFull = -8;

void* bz2_handle() {
  static void* h = dlopen("libbz2.so.1", RTLD_NOW | RTLD_LOCAL);
  return h;
}

bool bz2_decompress(const uint8_t* in, size_t in_len, std::vector<uint8_t>* out) {
  void* h = bz2_handle();
  auto fn = h ? (BzDecFn)dlsym(h, "BZ2_bzBuffToBuffDecompress") : nullptr;
  if (!fn || in_len > 0xFFFFFFFFu) return false;
  size_t cap = in_len * 8 < (1u << 20) ? (1u << 20) : in_len * 8;
  for (int tries = 0; tries < 8 && cap <= 0xFFFFFFFFu; ++tries, cap *= 4) {
    out->resize(cap);
    unsigned dl = (unsigned)cap;
    const int rc = fn((char*)out->data(), &dl, (char*)in, (unsigned)in_len, 0, 0);
    if (rc == kBzOk) {
      out->resize(dl);
      return true;
    }
    if (rc != kBzOutbuffFull) return false;
  }
  return false;
}

bool bz2_compress(const std::vector<uint8_t>& in, std::vector<uint8_t>* out) {
  void* h = bz2_handle();
  auto fn = h ? (BzEncFn)dlsym(h, "BZ2_bzBuffToBuffCompress") : nullptr;
  if (!fn) return false;
  unsigned dl = (unsigned)(in.size() + in.size() / 100 + 601);
  out->resize(dl);
  if (fn((char*)out->data(), &dl, (char*)in.data(), (unsigned)in.size(), 9, 0, 0) != kBzOk) return false;
  out->resize(dl);
  return true;
}

// ---- LZO1X decompressor (safe: bounds-checked) -------------------------------------------------
bool lzo1x_decompress(const uint8_t* in, size_t in_len, std::vector<uint8_t>* out) {
  const uint8_t* ip = in;
  const uint8_t* const ie = in + in_len;
  std::vector<uint8_t>& o = *out;
  o.clear();
  size_t t;
  auto need = [&](size_t n) { return (size_t)(ie - ip) >= n; };
  auto copy_lit = [&](size_t n) -> bool {
    if (!need(n)) return false;
    o.insert(o.end(), ip, ip + n);
    ip += n;
    return true;
  };
  auto copy_match = [&](size_t dist, size_t n) -> bool {
    if (dist == 0 || dist > o.size()) return false;
    size_t from = o.size() - dist;
    for (size_t k = 0; k < n; ++k) o.push_back(o[from + k]);
    return true;
  };
  auto lenext = [&](size_t base) -> long {  // zero-byte run length extension
    size_t v = 0;
    while (true) {
      if (!need(1)) return -1;
      if (*ip != 0) break;
      v += 255;
      ++ip;
      if (v > (1u << 30)) return -1;
    }
    return (long)(v + base + *ip++);
  };
  if (!need(1)) return false;
  int state = 0;  // 0: expect instruction; literals-after-match handled via trailing bits
  if (*ip > 17) {
    t = *ip++ - 17;
    if (!copy_lit(t)) return false;
    state = t < 4 ? 2 : 1;  // 2: after <4 literals (match follows), 1: after a literal run
  }
  while (true) {
    if (!need(1)) return false;
    t = *ip++;
    if (state == 0 && t < 16) {  // literal run
      if (t == 0) {
        long e = lenext(15);
        if (e < 0) return false;
        t = (size_t)e;
      }
      if (!copy_lit(t + 3)) return false;
      state = 1;
      continue;
    }
    size_t dist, len;
    if (t >= 64) {  // M2
      if (!need(1)) return false;
      dist = 1 + ((t >> 2) & 7) + ((size_t)(*ip++) << 3);
      len = (t >> 5) - 1 + 2;
    } else if (t >= 32) {  // M3
      t &= 31;
      if (t == 0) {
        long e = lenext(31);
        if (e < 0) return false;
        t = (size_t)e;
      }
      if (!need(2)) return false;
      dist = 1 + ((ip[0] | (ip[1] << 8)) >> 2);
      ip += 2;
      len = t + 2;
    } else if (t >= 16) {  // M4 (or end of stream)
      size_t hi = (t & 8) << 11;
      t &= 7;
      if (t == 0) {
        long e = lenext(7);
        if (e < 0) return false;
        t = (size_t)e;
      }
      if (!need(2)) return false;
      const size_t lo = (ip[0] | (ip[1] << 8)) >> 2;
      ip += 2;
      if (hi == 0 && lo == 0) return ip == ie;  // EOF marker
      dist = hi + lo + 0x4000;
      len = t + 2;
    } else {  // t < 16 after a literal run / match: short M1
      if (!need(1)) return false;
      if (state == 1) {
        dist = 1 + 0x0800 + (t >> 2) + ((size_t)(*ip++) << 2);
        len = 3;
      } else {
        dist = 1 + (t >> 2) + ((size_t)(*ip++) << 2);
        len = 2;
      }
    }
    if (!copy_match(dist, len)) return false;
    // trailing literals encoded in the low 2 bits of the byte two positions back
    t = ip[-2] & 3;
    if (t == 0) {
      state = 0;
      continue;
    }
    if (!copy_lit(t)) return false;
    state = 2;
  }
}

// ---- LZ4 block decompressor --------------------------------------------------------------------
bool lz4_decompress(const uint8_t* in, size_t in_len, std::vector<uint8_t>* out) {
  const uint8_t* ip = in;
  const uint8_t* ie = in + in_len;
  std::vector<uint8_t>& o = *out;
  o.clear();
  while (ip < ie) {
    const uint8_t tok = *ip++;
    size_t lit = tok >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (ip >= ie) return false;
        b = *ip++;
        lit += b;
      } while (b == 255);
    }
    if ((size_t)(ie - ip) < lit) return false;
    o.insert(o.end(), ip, ip + lit);
    ip += lit;
    if (ip >= ie) break;  // last sequence: literals only
    if (ie - ip < 2) return false;
    const size_t off = ip[0] | (ip[1] << 8);
    ip += 2;
    size_t ml = (tok & 15) + 4;
    if ((tok & 15) == 15) {
      uint8_t b;
      do {
        if (ip >= ie) return false;
        b = *ip++;
        ml += b;
      } while (b == 255);
    }
    if (off == 0 || off > o.size()) return false;
    const size_t from = o.size() - off;
    for (size_t k = 0; k < ml; ++k) o.push_back(o[from + k]);
  }
  return true;
}

struct Flow {
  int64_t first_ms, last_ms, received_ms;
  uint32_t sip, dip, rip;
  uint8_t v6, a6[32];  // IPv6 record: source (16 B) + destination (16 B) address, sip/dip = 0
  int32_t sport, dport, proto, flags, fwd, stos, dtos, dir, input, output, sas, das;
  int64_t ipkt, ibyt, opkt, obyt;
};

struct Handle {
  std::vector<Flow> flows;
  std::string err;
  int64_t blocks = 0, skipped_records = 0;
};

void decode_block(const uint8_t* b, size_t n, std::vector<std::vector<uint16_t>>* maps, Handle* h) {
  size_t pos = 0;
  while (pos + 4 <= n) {
    uint16_t type, size;
    std::memcpy(&type, b + pos, 2);
    std::memcpy(&size, b + pos + 2, 2);
    if (size < 4 || pos + size > n) break;
    const uint8_t* r = b + pos;
    if (type == 2 && size >= 10) {  // extension map
      uint16_t id;
      std::memcpy(&id, r + 4, 2);
      std::vector<uint16_t> ex;
      for (size_t o = 8; o + 2 <= size; o += 2) {
        uint16_t e;
        std::memcpy(&e, r + o, 2);
        if (e == 0) break;
        ex.push_back(e);
      }
      if (id >= maps->size()) maps->resize(id + 1);
      (*maps)[id] = ex;
    } else if (type == 10 && size >= 32) {
      Flow f;
      std::memset(&f, 0, sizeof f);
      uint16_t flags, ext_map, msf, msl, sp, dp;
      uint32_t first, last;
      std::memcpy(&flags, r + 4, 2);
      std::memcpy(&ext_map, r + 6, 2);
      std::memcpy(&msf, r + 8, 2);
      std::memcpy(&msl, r + 10, 2);
      std::memcpy(&first, r + 12, 4);
      std::memcpy(&last, r + 16, 4);
      f.fwd = r[20];
      f.flags = r[21];
      f.proto = r[22];
      f.stos = r[23];
      std::memcpy(&sp, r + 24, 2);
      std::memcpy(&dp, r + 26, 2);
      f.sport = sp;
      f.dport = dp;
      f.dir = r[30];
      f.first_ms = (int64_t)first * 1000 + msf;
      f.last_ms = (int64_t)last * 1000 + msl;
      size_t o = 32;
      if (flags & 1) {  // IPv6: carried verbatim (the pipeline keys v6 documents exactly)
        if (o + 32 > size) goto skip;
        f.v6 = 1;
        std::memcpy(f.a6, r + o, 32);
        f.sip = f.dip = 0;
        o += 32;
      } else {
        if (o + 8 > size) goto skip;
        std::memcpy(&f.sip, r + o, 4);
        std::memcpy(&f.dip, r + o + 4, 4);
        o += 8;
      }
      if (flags & 2) {
        if (o + 8 > size) goto skip;
        uint64_t v;
        std::memcpy(&v, r + o, 8);
        f.ipkt = (int64_t)v;
        o += 8;
      } else {
        uint32_t v;
        std::memcpy(&v, r + o, 4);
        f.ipkt = v;
        o += 4;
      }
      if (flags & 4) {
        if (o + 8 > size) goto skip;
        uint64_t v;
        std::memcpy(&v, r + o, 8);
        f.ibyt = (int64_t)v;
        o += 8;
      } else {
        if (o + 4 > size) goto skip;
        uint32_t v;
        std::memcpy(&v, r + o, 4);
        f.ibyt = v;
        o += 4;
      }
      if (ext_map < maps->size()) {
        for (uint16_t e : (*maps)[ext_map]) {
          const int es = ext_size(e);
          if (es == 0 || o + es > size) break;
          const uint8_t* x = r + o;
          uint16_t a16, b16;
          uint32_t a32, b32;
          uint64_t v64;
          switch (e) {
            case 4: std::memcpy(&a16, x, 2); std::memcpy(&b16, x + 2, 2); f.input = a16; f.output = b16; break;
            case 5: std::memcpy(&a32, x, 4); std::memcpy(&b32, x + 4, 4); f.input = (int32_t)a32; f.output = (int32_t)b32; break;
            case 6: std::memcpy(&a16, x, 2); std::memcpy(&b16, x + 2, 2); f.sas = a16; f.das = b16; break;
            case 7: std::memcpy(&a32, x, 4); std::memcpy(&b32, x + 4, 4); f.sas = (int32_t)a32; f.das = (int32_t)b32; break;
            case 8: f.dtos = x[0]; f.dir = x[1]; break;
            case 14: std::memcpy(&a32, x, 4); f.opkt = a32; break;
            case 15: std::memcpy(&v64, x, 8); f.opkt = (int64_t)v64; break;
            case 16: std::memcpy(&a32, x, 4); f.obyt = a32; break;
            case 17: std::memcpy(&v64, x, 8); f.obyt = (int64_t)v64; break;
            case 23: std::memcpy(&f.rip, x, 4); break;
            case 27: std::memcpy(&v64, x, 8); f.received_ms = (int64_t)v64; break;
            default: break;
          }
          o += es;
        }
      }
      if (f.received_ms == 0) f.received_ms = f.first_ms;
      h->flows.push_back(f);
      pos += size;
      continue;
    skip:
      ++h->skipped_records;
    } else {
      ++h->skipped_records;
    }
    pos += size;
  }
}

}  // namespace

ONI_NATIVE_API void* oni_nfcapd_open(const char* path) {
  auto* h = new Handle();
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    h->err = "cannot open";
    return h;
  }
  std::vector<uint8_t> buf;
  {
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    buf.resize(n > 0 ? (size_t)n : 0);
    if (n > 0 && std::fread(buf.data(), 1, buf.size(), f) != buf.size()) h->err = "short read";
    std::fclose(f);
  }
  if (!h->err.empty()) return h;
  if (buf.size() < 140 + 144) {
    h->err = "too short";
    return h;
  }
  uint16_t magic, version;
  uint32_t flags, nblocks;
  std::memcpy(&magic, buf.data(), 2);
  std::memcpy(&version, buf.data() + 2, 2);
  std::memcpy(&flags, buf.data() + 4, 4);
  std::memcpy(&nblocks, buf.data() + 8, 4);
  if (magic != kMagic || version != 1) {
    h->err = "not an nfcapd LAYOUT_VERSION_1 file";
    return h;
  }
  if ((flags & kFlagBZ2) && !bz2_handle()) {
    h->err = "bz2-compressed nfcapd file but libbz2.so.1 is not loadable";
    return h;
  }
  size_t pos = 140 + 160;  // header + stat record
  std::vector<std::vector<uint16_t>> maps;
  std::vector<uint8_t> dec;
  for (uint32_t bi = 0; bi < nblocks && pos + 12 <= buf.size(); ++bi) {
    uint32_t nrec, size;
    uint16_t id;
    std::memcpy(&nrec, buf.data() + pos, 4);
    std::memcpy(&size, buf.data() + pos + 4, 4);
    std::memcpy(&id, buf.data() + pos + 8, 2);
    pos += 12;
    if (pos + size > buf.size()) {
      h->err = "truncated block";
      break;
    }
    const uint8_t* data = buf.data() + pos;
    size_t dlen = size;
    if (id == 2) {
      if (flags & kFlagLZO) {
        if (!lzo1x_decompress(data, size, &dec)) {
          h->err = "lzo decompression failed";
          break;
        }
        data = dec.data();
        dlen = dec.size();
      } else if (flags & kFlagLZ4) {
        if (!lz4_decompress(data, size, &dec)) {
          h->err = "lz4 decompression failed";
          break;
        }
        data = dec.data();
        dlen = dec.size();
      } else if (flags & kFlagBZ2) {
        if (!bz2_decompress(data, size, &dec)) {
          h->err = "bz2 decompression failed";
          break;
        }
        data = dec.data();
        dlen = dec.size();
      }
      decode_block(data, dlen, &maps, h);
      ++h->blocks;
    }
    pos += size;
  }
  return h;
}

ONI_NATIVE_API int oni_nfcapd_info(void* hp, int64_t* n_flows, int64_t* blocks, int64_t* skipped, char* err,
                                   int err_len) {
  auto* h = (Handle*)hp;
  *n_flows = (int64_t)h->flows.size();
  *blocks = h->blocks;
  *skipped = h->skipped_records;
  std::snprintf(err, err_len, "%s", h->err.c_str());
  return h->err.empty() ? 0 : 1;
}

// out_i64: [n][8] first_ms,last_ms,received_ms,ipkt,ibyt,opkt,obyt,unused
// out_i32: [n][14] sport,dport,proto,flags,fwd,stos,dtos,dir,input,output,sas,das,sip,dip  (+ rip in out_rip)
ONI_NATIVE_API int oni_nfcapd_fetch(void* hp, int64_t* out_i64, int32_t* out_i32, uint32_t* out_rip) {
  auto* h = (Handle*)hp;
  for (size_t i = 0; i < h->flows.size(); ++i) {
    const Flow& f = h->flows[i];
    int64_t* a = out_i64 + i * 8;
    a[0] = f.first_ms; a[1] = f.last_ms; a[2] = f.received_ms; a[3] = f.ipkt; a[4] = f.ibyt; a[5] = f.opkt;
    a[6] = f.obyt; a[7] = 0;
    int32_t* b = out_i32 + i * 14;
    b[0] = f.sport; b[1] = f.dport; b[2] = f.proto; b[3] = f.flags; b[4] = f.fwd; b[5] = f.stos; b[6] = f.dtos;
    b[7] = f.dir; b[8] = f.input; b[9] = f.output; b[10] = f.sas; b[11] = f.das; b[12] = (int32_t)f.sip;
    b[13] = (int32_t)f.dip;
    out_rip[i] = f.rip;
  }
  return 0;
}

// IPv6 records: is_v6[n] (1 for IPv6 flows) and addrs[n][32] (source 16 B | destination 16 B)
ONI_NATIVE_API int oni_nfcapd_fetch_v6(void* hp, uint8_t* is_v6, uint8_t* addrs) {
  auto* h = (Handle*)hp;
  for (size_t i = 0; i < h->flows.size(); ++i) {
    const Flow& f = h->flows[i];
    is_v6[i] = f.v6;
    if (f.v6) std::memcpy(addrs + i * 32, f.a6, 32);
    else std::memset(addrs + i * 32, 0, 32);
  }
  return 0;
}

ONI_NATIVE_API void oni_nfcapd_free(void* hp) { delete (Handle*)hp; }

ONI_NATIVE_API int oni_lzo1x_decompress(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap, int64_t* out_len) {
  std::vector<uint8_t> o;
  if (!lzo1x_decompress(in, (size_t)n, &o)) return 1;
  if ((int64_t)o.size() > cap) return 2;
  std::memcpy(out, o.data(), o.size());
  *out_len = (int64_t)o.size();
  return 0;
}

ONI_NATIVE_API int oni_lz4_decompress(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap, int64_t* out_len) {
  std::vector<uint8_t> o;
  if (!lz4_decompress(in, (size_t)n, &o)) return 1;
  if ((int64_t)o.size() > cap) return 2;
  std::memcpy(out, o.data(), o.size());
  *out_len = (int64_t)o.size();
  return 0;
}

// ---- writer: LAYOUT_VERSION_1, one ext map {4 (io16), 6 (as16), 8 (multiple), 14, 16, 23, 27} ----
// compression: 0 none, 1 LZO1X (literal-run encoding: valid stream, no matches), 2 LZ4 (literals only),
// 3 bzip2 (libbz2)
ONI_NATIVE_API int64_t oni_nfcapd_write(const char* path, int64_t n, const int64_t* first_ms, const int64_t* last_ms,
                                        const int64_t* received_ms, const uint32_t* sip, const uint32_t* dip,
                                        const int32_t* sport, const int32_t* dport, const int32_t* proto,
                                        const int32_t* tflags, const int64_t* ipkt, const int64_t* ibyt,
                                        const int64_t* opkt, const int64_t* obyt, const int32_t* input,
                                        const int32_t* output, const int32_t* sas, const int32_t* das,
                                        const uint32_t* rip, const uint8_t* is_v6, const uint8_t* addrs6,
                                        int compression, int per_block) {
  FILE* f = std::fopen(path, "wb");
  if (!f) return -1;
  std::vector<uint8_t> hdr(140 + 160, 0);
  const uint16_t magic = kMagic, version = 1;
  const uint32_t flags =
      compression == 1 ? kFlagLZO : (compression == 2 ? kFlagLZ4 : (compression == 3 ? kFlagBZ2 : 0));
  if (compression == 3 && !bz2_handle()) {
    std::fclose(f);
    return -2;
  }
  const uint32_t nblocks = (uint32_t)((n + per_block - 1) / per_block) + 1;
  std::memcpy(hdr.data(), &magic, 2);
  std::memcpy(hdr.data() + 2, &version, 2);
  std::memcpy(hdr.data() + 4, &flags, 4);
  std::memcpy(hdr.data() + 8, &nblocks, 4);
  std::snprintf((char*)hdr.data() + 12, 128, "oni355");
  const uint64_t nf = (uint64_t)n;
  std::memcpy(hdr.data() + 140, &nf, 8);
  std::fwrite(hdr.data(), 1, hdr.size(), f);
  auto put_block = [&](const std::vector<uint8_t>& raw, uint32_t nrec) {
    std::vector<uint8_t> payload;
    if (compression == 1) {
      // LZO1X literal-only stream: ONE literal run (a run may not follow a run), then EOF.
      // Short blocks use the first-byte "t + 17" form, longer ones the zero-extended run length.
      const size_t len = raw.size();
      if (len <= 238) {
        payload.push_back((uint8_t)(len + 17));
      } else {
        size_t t = len - 3;
        if (t <= 15) {
          payload.push_back((uint8_t)t);
        } else {
          payload.push_back(0);
          t -= 15;
          while (t > 255) {
            payload.push_back(0);
            t -= 255;
          }
          payload.push_back((uint8_t)t);
        }
      }
      payload.insert(payload.end(), raw.begin(), raw.end());
      payload.push_back(17);  // M4 EOF: 0x11 0x00 0x00
      payload.push_back(0);
      payload.push_back(0);
    } else if (compression == 2) {
      size_t lit = raw.size();
      if (lit >= 15) {
        payload.push_back(0xF0);
        size_t rem = lit - 15;
        while (rem >= 255) {
          payload.push_back(255);
          rem -= 255;
        }
        payload.push_back((uint8_t)rem);
      } else {
        payload.push_back((uint8_t)(lit << 4));
      }
      payload.insert(payload.end(), raw.begin(), raw.end());
    } else if (compression == 3) {
      if (!bz2_compress(raw, &payload)) payload.clear();
    } else {
      payload = raw;
    }
    const uint32_t size = (uint32_t)payload.size();
    const uint16_t id = 2, bflags = 0;
    std::fwrite(&nrec, 4, 1, f);
    std::fwrite(&size, 4, 1, f);
    std::fwrite(&id, 2, 1, f);
    std::fwrite(&bflags, 2, 1, f);
    std::fwrite(payload.data(), 1, payload.size(), f);
  };
  // block 0: extension map
  {
    std::vector<uint8_t> m;
    const uint16_t ex[] = {4, 6, 8, 14, 16, 23, 27, 0};
    const uint16_t type = 2, size = (uint16_t)(8 + sizeof(ex)), map_id = 0;
    uint16_t ext_total = 0;
    for (uint16_t e : ex) ext_total += (uint16_t)ext_size(e);
    m.resize(size);
    std::memcpy(m.data(), &type, 2);
    std::memcpy(m.data() + 2, &size, 2);
    std::memcpy(m.data() + 4, &map_id, 2);
    std::memcpy(m.data() + 6, &ext_total, 2);
    std::memcpy(m.data() + 8, ex, sizeof(ex));
    put_block(m, 1);
  }
  std::vector<uint8_t> raw;
  uint32_t nrec = 0;
  for (int64_t i = 0; i < n; ++i) {
    const bool v6 = is_v6 && addrs6 && is_v6[i];
    const uint16_t type = 10, size = (uint16_t)(32 + (v6 ? 32 : 8) + 8 + 8 + 4 + 4 + 4 + 8 + 8 + 4 + 8);
    uint8_t r[32 + 32 + 8 + 8 + 4 + 4 + 4 + 8 + 8 + 4 + 8];
    std::memset(r, 0, size);
    const uint16_t fl = (uint16_t)(2 | 4 | (v6 ? 1 : 0)), ext = 0, msf = (uint16_t)(first_ms[i] % 1000), msl = (uint16_t)(last_ms[i] % 1000);
    const uint32_t first = (uint32_t)(first_ms[i] / 1000), last = (uint32_t)(last_ms[i] / 1000);
    std::memcpy(r, &type, 2);
    std::memcpy(r + 2, &size, 2);
    std::memcpy(r + 4, &fl, 2);
    std::memcpy(r + 6, &ext, 2);
    std::memcpy(r + 8, &msf, 2);
    std::memcpy(r + 10, &msl, 2);
    std::memcpy(r + 12, &first, 4);
    std::memcpy(r + 16, &last, 4);
    r[21] = (uint8_t)tflags[i];
    r[22] = (uint8_t)proto[i];
    const uint16_t sp = (uint16_t)sport[i], dp = (uint16_t)dport[i];
    std::memcpy(r + 24, &sp, 2);
    std::memcpy(r + 26, &dp, 2);
    size_t o = 32;
    if (v6) {
      std::memcpy(r + o, addrs6 + i * 32, 32);
      o += 32;
    } else {
      std::memcpy(r + o, &sip[i], 4);
      std::memcpy(r + o + 4, &dip[i], 4);
      o += 8;
    }
    const uint64_t pk = (uint64_t)ipkt[i], by = (uint64_t)ibyt[i];
    std::memcpy(r + o, &pk, 8);
    std::memcpy(r + o + 8, &by, 8);
    o += 16;
    const uint16_t in16 = (uint16_t)input[i], out16 = (uint16_t)output[i], sa = (uint16_t)sas[i], da = (uint16_t)das[i];
    std::memcpy(r + o, &in16, 2); std::memcpy(r + o + 2, &out16, 2); o += 4;
    std::memcpy(r + o, &sa, 2); std::memcpy(r + o + 2, &da, 2); o += 4;
    o += 4;  // ext 8: dst_tos, dir, masks
    const uint32_t op = (uint32_t)opkt[i], ob = (uint32_t)obyt[i];
    std::memcpy(r + o, &op, 4); o += 4;
    std::memcpy(r + o, &ob, 4); o += 4;
    std::memcpy(r + o, &rip[i], 4); o += 4;
    const uint64_t rcv = (uint64_t)received_ms[i];
    std::memcpy(r + o, &rcv, 8);
    raw.insert(raw.end(), r, r + size);
    if (++nrec == (uint32_t)per_block || i == n - 1) {
      put_block(raw, nrec);
      raw.clear();
      nrec = 0;
    }
  }
  std::fclose(f);
  return n;
}
