// DNS-response decoder for pcap / pcapng captures -- replaces the reference's
// `editcap -c <pkt_num>` split + `tshark -T fields -e frame.time -e frame.time_epoch -e frame.len
// -e ip.src -e ip.dst -e dns.resp.name -e dns.resp.type -e dns.resp.class -e dns.flags.rcode
// -e dns.a` pipeline (oni-ingest dns worker, SURVEY.md §2.2 C02, [U-M]).
//
// P4 (intra-file parallelism) without heuristics: one sequential pass hops over record headers to
// index every packet (cheap: 16-byte reads), then packets are decoded in parallel (OpenMP over
// index ranges) into thread-local column buffers that are concatenated in order.
//
// Supported: classic pcap (µs / ns, either byte order), pcapng (SHB/IDB/EPB/SPB/OPB);
// link types Ethernet (VLAN/QinQ), raw IPv4/IPv6, Linux cooked (SLL, SLL2), NULL/loopback;
// IPv4 (fragmented datagrams reassembled in a serial pass after the parallel decode) and IPv6 (no
// extension headers); DNS over UDP from port 53 and over TCP from port 53 (every complete
// length-prefixed message inside a segment); DNS header + first question (with name-compression
// pointers) + A answers.
#include <fcntl.h>
#include <omp.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <ctime>
#include <string>
#include <map>
#include <tuple>
#include <vector>

#include "../native/oni_native.h"

namespace {

struct Pkt {
  size_t off;    // start of packet bytes
  uint32_t caplen, origlen;
  int64_t ts_ns;
  int linktype;
};

inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
inline uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
inline uint32_t rd32(const uint8_t* p, bool swap) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return swap ? __builtin_bswap32(v) : v;
}
inline uint16_t rd16(const uint8_t* p, bool swap) {
  uint16_t v;
  std::memcpy(&v, p, 2);
  return swap ? __builtin_bswap16(v) : v;
}

bool index_pcap(const uint8_t* b, size_t n, std::vector<Pkt>* out, std::string* err) {
  if (n < 24) {
    *err = "file too short";
    return false;
  }
  const uint32_t magic = *(const uint32_t*)b;
  bool swap = false, nano = false;
  if (magic == 0xa1b2c3d4u) {
  } else if (magic == 0xd4c3b2a1u) {
    swap = true;
  } else if (magic == 0xa1b23c4du) {
    nano = true;
  } else if (magic == 0x4d3cb2a1u) {
    swap = nano = true;
  } else if (magic == 0x0a0d0d0au) {
    // pcapng
    std::vector<int> if_link;
    std::vector<int64_t> if_tsres;  // ticks per second
    size_t pos = 0;
    bool sw = false;
    while (pos + 12 <= n) {
      uint32_t type = rd32(b + pos, sw);
      if (type == 0x0a0d0d0au) {
        const uint32_t bom = *(const uint32_t*)(b + pos + 8);
        sw = (bom == 0x4d3c2b1au);
        if_link.clear();
        if_tsres.clear();
      }
      const uint32_t blen = rd32(b + pos + 4, sw);
      if (blen < 12 || pos + blen > n) break;
      if (type == 1) {  // IDB
        if_link.push_back(rd16(b + pos + 8, sw));
        int64_t res = 1000000;
        size_t o = pos + 16;
        while (o + 4 <= pos + blen - 4) {
          const uint16_t code = rd16(b + o, sw), len = rd16(b + o + 2, sw);
          if (code == 0) break;
          if (code == 9 && len >= 1) {
            const uint8_t r = b[o + 4];
            res = 1;
            if (r & 0x80)
              for (int i = 0; i < (r & 0x7f); ++i) res *= 2;
            else
              for (int i = 0; i < r; ++i) res *= 10;
          }
          o += 4 + ((len + 3) & ~3u);
        }
        if_tsres.push_back(res);
      } else if (type == 6 || type == 3 || type == 2) {  // EPB / SPB / OPB
        Pkt p;
        if (type == 3) {
          p.origlen = rd32(b + pos + 8, sw);
          p.caplen = blen - 16 < p.origlen ? blen - 16 : p.origlen;
          p.off = pos + 12;
          p.ts_ns = 0;
          p.linktype = if_link.empty() ? 1 : if_link[0];
        } else {
          const uint32_t ifid = type == 6 ? rd32(b + pos + 8, sw) : rd16(b + pos + 8, sw);
          const uint64_t ts = ((uint64_t)rd32(b + pos + 12, sw) << 32) | rd32(b + pos + 16, sw);
          p.caplen = rd32(b + pos + 20, sw);
          p.origlen = rd32(b + pos + 24, sw);
          p.off = pos + 28;
          const int64_t res = ifid < if_tsres.size() ? if_tsres[ifid] : 1000000;
          p.ts_ns = (int64_t)((ts / (uint64_t)res) * 1000000000ull + (ts % (uint64_t)res) * (1000000000ull / (uint64_t)res));
          p.linktype = ifid < if_link.size() ? if_link[ifid] : 1;
        }
        if (p.off + p.caplen <= pos + blen) out->push_back(p);
      }
      pos += blen;
    }
    return true;
  } else {
    *err = "not a pcap/pcapng file";
    return false;
  }
  const int link = (int)(rd32(b + 20, swap) & 0x0FFFFFFF);
  size_t pos = 24;
  while (pos + 16 <= n) {
    Pkt p;
    const uint32_t sec = rd32(b + pos, swap), frac = rd32(b + pos + 4, swap);
    p.caplen = rd32(b + pos + 8, swap);
    p.origlen = rd32(b + pos + 12, swap);
    p.off = pos + 16;
    if (p.caplen > 262144 || p.off + p.caplen > n) break;  // truncated tail
    p.ts_ns = (int64_t)sec * 1000000000ll + (nano ? frac : (int64_t)frac * 1000);
    p.linktype = link;
    out->push_back(p);
    pos = p.off + p.caplen;
  }
  return true;
}

// ---- parallel index of a classic pcap -------------------------------------------------------------
// Walking classic pcap records is a dependent-load chain (each header's caplen gives the next
// offset): ~25 ns per record, 50 ms for a 2M-packet day on one core. Here T threads each take a
// byte range; thread t > 0 SPECULATES its first record start -- the first offset from which
// kChain consecutive headers are plausible and chain exactly -- and walks records while they start
// inside its range. The stitch is exact: range t's records are accepted only if its first record is
// the offset where range t − 1's walk left off (the sequential walk from byte 24); otherwise the
// range is re-walked from that offset. Speculation only decides how much is re-walked.
struct ClassicHdr {
  bool swap, nano;
  int link;
  uint32_t sec0;  // first record's seconds (plausibility window for speculation)
};

struct IdxPart {
  std::vector<Pkt> pk;
  size_t first = 0;     // offset of the first record walked (SIZE_MAX: none found)
  size_t landing = 0;   // offset after the last record walked (next record start)
  bool broke = false;   // the walk hit a truncated / invalid record (the sequential walk ends there)
};

constexpr int kChain = 6;

inline bool classic_hdr_ok(const uint8_t* b, size_t n, size_t pos, const ClassicHdr& h, bool strict) {
  if (pos + 16 > n) return false;
  const uint32_t caplen = rd32(b + pos + 8, h.swap);
  if (caplen > 262144 || pos + 16 + caplen > n) return false;
  if (!strict) return true;
  const uint32_t sec = rd32(b + pos, h.swap), frac = rd32(b + pos + 4, h.swap);
  const uint32_t origlen = rd32(b + pos + 12, h.swap);
  if (frac >= (h.nano ? 1000000000u : 1000000u) || origlen < caplen || origlen > 262144) return false;
  const int64_t dsec = (int64_t)sec - (int64_t)h.sec0;
  return dsec > -864000 && dsec < 864000;  // within 10 days of the first record
}

// walk records from `pos` while they start before `end` (the sequential walk's rule)
void walk_classic(const uint8_t* b, size_t n, size_t pos, size_t end, const ClassicHdr& h, IdxPart* part) {
  part->first = pos;
  while (pos < end && pos + 16 <= n) {
    Pkt p;
    const uint32_t sec = rd32(b + pos, h.swap), frac = rd32(b + pos + 4, h.swap);
    p.caplen = rd32(b + pos + 8, h.swap);
    p.origlen = rd32(b + pos + 12, h.swap);
    p.off = pos + 16;
    if (p.caplen > 262144 || p.off + p.caplen > n) {
      part->broke = true;
      break;
    }
    p.ts_ns = (int64_t)sec * 1000000000ll + (h.nano ? frac : (int64_t)frac * 1000);
    p.linktype = h.link;
    part->pk.push_back(p);
    pos = p.off + p.caplen;
  }
  if (pos + 16 > n && pos < end) part->broke = true;  // the file ends inside this range
  part->landing = pos;
}

// first offset in [lo, hi) from which kChain plausible headers chain (or reach EOF exactly)
size_t speculate_start(const uint8_t* b, size_t n, size_t lo, size_t hi, const ClassicHdr& h) {
  for (size_t o = lo; o < hi; ++o) {
    size_t q = o;
    int k = 0;
    for (; k < kChain; ++k) {
      if (q == n) break;  // the chain reaches the end of the file exactly
      if (!classic_hdr_ok(b, n, q, h, true)) break;
      q += 16 + rd32(b + q + 8, h.swap);
    }
    if (k == kChain || q == n) return o;
  }
  return SIZE_MAX;
}

// per-range record lists whose concatenation is exactly the sequential walk from byte 24
std::vector<IdxPart> index_classic_parallel(const uint8_t* b, size_t n, const ClassicHdr& h, int T) {
  std::vector<IdxPart> parts(T);
  std::vector<size_t> lo(T + 1);
  for (int t = 0; t <= T; ++t) lo[t] = t == 0 ? 24 : (t == T ? n : 24 + (n - 24) * (size_t)t / T);
#pragma omp parallel for num_threads(T) schedule(static, 1)
  for (int t = 0; t < T; ++t) {
    const size_t start = t == 0 ? 24 : speculate_start(b, n, lo[t], lo[t + 1], h);
    if (start == SIZE_MAX) {
      parts[t].first = SIZE_MAX;
      continue;
    }
    walk_classic(b, n, start, lo[t + 1], h, &parts[t]);
  }
  // exact stitch
  size_t pos = 24;
  bool ended = false;
  for (int t = 0; t < T; ++t) {
    IdxPart& p = parts[t];
    if (ended) {
      p.pk.clear();
      continue;
    }
    if (pos >= lo[t + 1]) {  // the previous range's last record already covers this range
      p.pk.clear();
      continue;
    }
    if (p.first != pos) {  // speculation missed: re-walk from where the sequential walk stands
      IdxPart q;
      walk_classic(b, n, pos, lo[t + 1], h, &q);
      p = std::move(q);
    }
    pos = p.landing;
    ended = p.broke;
  }
  return parts;
}

// read a (possibly compressed) DNS name at `o`, appending it to `out` when given (nothing is
// appended on failure); returns bytes consumed at o, or -1. No allocation: the decoder calls this
// for every packet, so names go straight into the thread's column buffer.
int read_name(const uint8_t* m, size_t mlen, size_t o, std::string* out) {
  const size_t base = out ? out->size() : 0;
  size_t pos = o, len = 0;
  int consumed = -1;
  int jumps = 0;
  while (pos < mlen) {
    const uint8_t l = m[pos];
    if (l == 0) {
      if (consumed < 0) consumed = (int)(pos + 1 - o);
      return consumed;
    }
    if ((l & 0xC0) == 0xC0) {
      if (pos + 1 >= mlen || ++jumps > 32) break;
      if (consumed < 0) consumed = (int)(pos + 2 - o);
      pos = ((size_t)(l & 0x3F) << 8) | m[pos + 1];
      continue;
    }
    if ((l & 0xC0) != 0 || pos + 1 + l > mlen) break;
    len += (len ? 1 : 0) + l;
    if (len > 255) break;
    if (out) {
      if (out->size() > base) out->push_back('.');
      out->append((const char*)m + pos + 1, l);
    }
    pos += 1 + l;
  }
  if (out) out->resize(base);
  return -1;
}

// dotted IPv4 text appended without snprintf
void put_ipv4(std::string* s, const uint8_t* a) {
  for (int k = 0; k < 4; ++k) {
    if (k) s->push_back('.');
    const unsigned v = a[k];
    if (v >= 100) s->push_back((char)('0' + v / 100));
    if (v >= 10) s->push_back((char)('0' + (v / 10) % 10));
    s->push_back((char)('0' + v % 10));
  }
}

struct Frag {
  uint32_t src, dst, off;
  uint16_t id;
  uint8_t proto;
  bool more;
  int64_t ts_ns, pkt;
  uint32_t origlen;
  std::vector<uint8_t> data;
};

struct Rows {
  std::vector<int64_t> ts_ns;
  std::vector<int32_t> frame_len, qtype, qclass, rcode;
  std::vector<uint32_t> ip_src, ip_dst;
  std::vector<int64_t> name_end, a_end;  // running offsets into chars
  std::vector<int64_t> pkt;              // packet index of each row (packet order)
  std::string names, as;
  std::vector<Frag> frags;               // IPv4 fragments seen by this thread
  int64_t tcp_partial = 0, frag_incomplete = 0;
};

// append rows [0, src.size) of `s` to `a` (offsets rebased)
void append_rows(Rows& a, const Rows& s) {
  const int64_t nb = (int64_t)a.names.size(), ab = (int64_t)a.as.size();
  a.ts_ns.insert(a.ts_ns.end(), s.ts_ns.begin(), s.ts_ns.end());
  a.frame_len.insert(a.frame_len.end(), s.frame_len.begin(), s.frame_len.end());
  a.ip_src.insert(a.ip_src.end(), s.ip_src.begin(), s.ip_src.end());
  a.ip_dst.insert(a.ip_dst.end(), s.ip_dst.begin(), s.ip_dst.end());
  a.qtype.insert(a.qtype.end(), s.qtype.begin(), s.qtype.end());
  a.qclass.insert(a.qclass.end(), s.qclass.begin(), s.qclass.end());
  a.rcode.insert(a.rcode.end(), s.rcode.begin(), s.rcode.end());
  a.pkt.insert(a.pkt.end(), s.pkt.begin(), s.pkt.end());
  for (auto e : s.name_end) a.name_end.push_back(e + nb);
  for (auto e : s.a_end) a.a_end.push_back(e + ab);
  a.names += s.names;
  a.as += s.as;
  a.tcp_partial += s.tcp_partial;
  a.frag_incomplete += s.frag_incomplete;
}

// rows in packet order (reassembled datagrams were appended after the parallel pass)
Rows packet_order(const Rows& a) {
  const size_t n = a.ts_ns.size();
  std::vector<size_t> o(n);
  for (size_t i = 0; i < n; ++i) o[i] = i;
  std::stable_sort(o.begin(), o.end(), [&](size_t x, size_t y) { return a.pkt[x] < a.pkt[y]; });
  Rows b;
  b.tcp_partial = a.tcp_partial;
  b.frag_incomplete = a.frag_incomplete;
  for (size_t k = 0; k < n; ++k) {
    const size_t i = o[k];
    b.ts_ns.push_back(a.ts_ns[i]);
    b.frame_len.push_back(a.frame_len[i]);
    b.ip_src.push_back(a.ip_src[i]);
    b.ip_dst.push_back(a.ip_dst[i]);
    b.qtype.push_back(a.qtype[i]);
    b.qclass.push_back(a.qclass[i]);
    b.rcode.push_back(a.rcode[i]);
    b.pkt.push_back(a.pkt[i]);
    const int64_t n0 = i ? a.name_end[i - 1] : 0, a0 = i ? a.a_end[i - 1] : 0;
    b.names.append(a.names, (size_t)n0, (size_t)(a.name_end[i] - n0));
    b.as.append(a.as, (size_t)a0, (size_t)(a.a_end[i] - a0));
    b.name_end.push_back((int64_t)b.names.size());
    b.a_end.push_back((int64_t)b.as.size());
  }
  return b;
}

uint32_t fold_ipv6(const uint8_t* a) {
  uint32_t h = 2166136261u;
  for (int i = 0; i < 16; ++i) h = (h ^ a[i]) * 16777619u;
  return h;
}

// one DNS message (UDP payload, or one length-prefixed TCP message) → a row (responses only)
void parse_dns(const uint8_t* m, size_t ml, int64_t ts_ns, uint32_t origlen, uint32_t src, uint32_t dst, int64_t pkt,
               Rows* r) {
  if (ml < 12) return;
  const uint16_t flags = be16(m + 2);
  if (!(flags & 0x8000)) return;  // responses only
  const int qd = be16(m + 4), an = be16(m + 6);
  if (qd < 1) return;
  const size_t name0 = r->names.size(), a0 = r->as.size();
  int c = read_name(m, ml, 12, &r->names);
  if (c < 0 || (size_t)(12 + c + 4) > ml) {
    r->names.resize(name0);
    return;
  }
  size_t pos = 12 + c;
  const int qtype = be16(m + pos), qclass = be16(m + pos + 2);
  pos += 4;
  for (int q = 1; q < qd; ++q) {  // skip further questions
    int cc = read_name(m, ml, pos, nullptr);
    if (cc < 0) {
      r->names.resize(name0);
      return;
    }
    pos += cc + 4;
  }
  for (int a = 0; a < an && pos < ml; ++a) {
    int cc = read_name(m, ml, pos, nullptr);
    if (cc < 0 || pos + cc + 10 > ml) break;
    pos += cc;
    const int type = be16(m + pos), rdlen = be16(m + pos + 8);
    pos += 10;
    if (pos + rdlen > ml) break;
    if (type == 1 && rdlen == 4) {
      if (r->as.size() > a0) r->as.push_back(',');
      put_ipv4(&r->as, m + pos);
    }
    pos += rdlen;
  }
  r->ts_ns.push_back(ts_ns);
  r->frame_len.push_back((int32_t)origlen);
  r->ip_src.push_back(src);
  r->ip_dst.push_back(dst);
  r->qtype.push_back(qtype);
  r->qclass.push_back(qclass);
  r->rcode.push_back(flags & 0x000F);
  r->name_end.push_back((int64_t)r->names.size());
  r->a_end.push_back((int64_t)r->as.size());
  r->pkt.push_back(pkt);
}

// transport payload → DNS messages: UDP from port 53 (one message); TCP from port 53 (every
// complete 2-byte-length-prefixed message inside this segment; messages split across segments
// would need stream reassembly and are counted in Rows::tcp_partial instead)
void parse_transport(const uint8_t* t, size_t tl, int proto, int64_t ts_ns, uint32_t origlen, uint32_t src,
                     uint32_t dst, int64_t pkt, Rows* r) {
  if (proto == 17) {
    if (tl < 8 || be16(t) != 53) return;
    parse_dns(t + 8, tl - 8, ts_ns, origlen, src, dst, pkt, r);
  } else if (proto == 6) {
    if (tl < 20 || be16(t) != 53) return;
    const size_t hl = (size_t)(t[12] >> 4) * 4;
    if (hl < 20 || hl > tl) return;
    size_t o = hl;
    while (o + 2 <= tl) {
      const size_t len = be16(t + o);
      if (len == 0) break;
      if (o + 2 + len > tl) {
        ++r->tcp_partial;
        break;
      }
      parse_dns(t + o + 2, len, ts_ns, origlen, src, dst, pkt, r);
      o += 2 + len;
    }
  }
}

void decode(const uint8_t* base, const Pkt& p, int64_t pkt, Rows* r) {
  const uint8_t* d = base + p.off;
  size_t n = p.caplen, o = 0;
  int ethertype = 0;
  switch (p.linktype) {
    case 1:  // Ethernet
      if (n < 14) return;
      ethertype = be16(d + 12);
      o = 14;
      while ((ethertype == 0x8100 || ethertype == 0x88a8) && o + 4 <= n) {
        ethertype = be16(d + o + 2);
        o += 4;
      }
      break;
    case 113:  // Linux SLL
      if (n < 16) return;
      ethertype = be16(d + 14);
      o = 16;
      break;
    case 276:  // Linux SLL2
      if (n < 20) return;
      ethertype = be16(d);
      o = 20;
      break;
    case 0:  // NULL / loopback (host order family)
      if (n < 4) return;
      ethertype = (d[0] == 2 || d[3] == 2) ? 0x0800 : 0x86DD;
      o = 4;
      break;
    default:  // raw IP (101, 228, 229, 12, 14)
      if (n < 1) return;
      ethertype = (d[0] >> 4) == 6 ? 0x86DD : 0x0800;
      o = 0;
  }
  if (ethertype == 0x0800) {
    if (o + 20 > n) return;
    const int ihl = (d[o] & 0x0F) * 4;
    const int proto = d[o + 9];
    if ((d[o] >> 4) != 4 || ihl < 20 || o + ihl > n || (proto != 17 && proto != 6)) return;
    const uint32_t src = be32(d + o + 12), dst = be32(d + o + 16);
    const uint16_t ff = be16(d + o + 6);
    size_t end = o + be16(d + o + 2);  // IP total length bounds the payload (Ethernet padding)
    if (end > n || end < o + ihl) end = n;
    if ((ff & 0x3FFF) != 0) {  // IPv4 fragment: kept for the serial reassembly pass
      Frag f;
      f.src = src;
      f.dst = dst;
      f.id = be16(d + o + 4);
      f.proto = (uint8_t)proto;
      f.off = (uint32_t)(ff & 0x1FFF) * 8u;
      f.more = (ff & 0x2000) != 0;
      f.ts_ns = p.ts_ns;
      f.origlen = p.origlen;
      f.pkt = pkt;
      f.data.assign(d + o + ihl, d + end);
      r->frags.push_back(std::move(f));
      return;
    }
    parse_transport(d + o + ihl, end - o - ihl, proto, p.ts_ns, p.origlen, src, dst, pkt, r);
  } else if (ethertype == 0x86DD) {
    if (o + 40 > n) return;
    const int nh = d[o + 6];
    if (nh != 17 && nh != 6) return;
    parse_transport(d + o + 40, n - o - 40, nh, p.ts_ns, p.origlen, fold_ipv6(d + o + 8), fold_ipv6(d + o + 24), pkt, r);
  }
}

// IPv4 fragment reassembly (RFC 791), in packet order. Fragments are grouped by (src, dst, id,
// proto) into OPEN datagrams; a datagram closes as soon as its pieces cover [0, end of the last
// (MF = 0) fragment) without a hole, and the row takes the frame time / length / index of the
// fragment that completed it (tshark's view). The 16-bit IP id wraps within a day-long capture, so
// a group is also closed (as incomplete) when a fragment offset it already holds shows up again with
// different bytes -- that is the next datagram with the same id (an exact duplicate of a held piece
// is dropped) -- or when the new fragment arrives more than
// kFragTimeoutNs of frame time after the group's first one (the kernel's ipfrag_time is 30 s).
constexpr int64_t kFragTimeoutNs = 30ll * 1000000000ll;

struct OpenDgram {
  std::vector<const Frag*> parts;
  int64_t first_ts = 0;
};

// complete? → parse into r and return true
bool try_complete(const OpenDgram& g, Rows* r) {
  size_t total = 0;
  bool last = false;
  const Frag* newest = g.parts[0];
  for (const Frag* f : g.parts) {
    if (!f->more) {
      last = true;
      total = f->off + f->data.size();
    }
    if (f->pkt > newest->pkt) newest = f;
  }
  if (!last || total > 65535) return false;
  std::vector<const Frag*> o(g.parts);
  std::stable_sort(o.begin(), o.end(), [](const Frag* a, const Frag* b) { return a->off < b->off; });
  size_t covered = 0;
  for (const Frag* f : o) {
    if (f->off > covered) return false;  // hole
    const size_t e = f->off + f->data.size();
    if (e > covered) covered = e;
  }
  if (covered < total) return false;
  std::vector<uint8_t> buf(total);
  for (const Frag* f : o) {
    const size_t e = f->off + f->data.size();
    if (e > f->off && f->off < total) std::memcpy(buf.data() + f->off, f->data.data(), std::min(e, total) - f->off);
  }
  const Frag& h = *o[0];
  parse_transport(buf.data(), total, h.proto, newest->ts_ns, newest->origlen, h.src, h.dst, newest->pkt, r);
  return true;
}

void reassemble(std::vector<Frag>& fr, Rows* r) {
  std::stable_sort(fr.begin(), fr.end(), [](const Frag& a, const Frag& b) { return a.pkt < b.pkt; });
  std::map<std::tuple<uint32_t, uint32_t, uint16_t, uint8_t>, OpenDgram> open;
  for (const Frag& f : fr) {
    const auto key = std::make_tuple(f.src, f.dst, f.id, f.proto);
    auto it = open.find(key);
    if (it != open.end()) {
      bool restart = f.ts_ns - it->second.first_ts > kFragTimeoutNs;
      bool duplicate = false;
      for (const Frag* p : it->second.parts) {
        if (p->off != f.off) continue;
        // an exact copy of a piece the group holds (mirror / SPAN captures duplicate packets) is
        // dropped, as tshark's reassembly does; a different payload at a held offset is the next
        // datagram reusing the id
        if (p->more == f.more && p->data == f.data) duplicate = true;
        else restart = true;
      }
      if (duplicate && !restart) continue;
      if (restart) {
        ++r->frag_incomplete;
        open.erase(it);
        it = open.end();
      }
    }
    if (it == open.end()) {
      it = open.emplace(key, OpenDgram{}).first;
      it->second.first_ts = f.ts_ns;
    }
    it->second.parts.push_back(&f);
    if (try_complete(it->second, r)) open.erase(it);
  }
  r->frag_incomplete += (int64_t)open.size();
}

struct Handle {
  std::vector<Rows> parts;  // per-thread rows in packet order (one part after a reassembly pass)
  int64_t packets = 0, rows = 0, name_bytes = 0, a_bytes = 0, tcp_partial = 0, frag_incomplete = 0;
  std::string err;
};

}  // namespace

ONI_NATIVE_API void* oni_pcap_dns_open(const char* path, int threads) {
  auto* h = new Handle();
  const int fd = ::open(path, O_RDONLY);
  if (fd < 0) {
    h->err = "cannot open";
    return h;
  }
  struct stat st;
  fstat(fd, &st);
  const size_t n = (size_t)st.st_size;
  const uint8_t* b = nullptr;
  // no MAP_POPULATE: the index threads fault their own ranges in parallel
  if (n) b = (const uint8_t*)mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
  const int T = threads > 0 ? threads : std::min(omp_get_max_threads(), 16);
  std::vector<std::vector<Pkt>> lists;  // per-range packet lists; their concatenation is packet order
  bool ok = b && b != MAP_FAILED && n >= 24;
  if (ok) {
    const uint32_t magic = *(const uint32_t*)b;
    const bool classic = magic == 0xa1b2c3d4u || magic == 0xd4c3b2a1u || magic == 0xa1b23c4du || magic == 0x4d3cb2a1u;
    if (classic) {
      ClassicHdr hh;
      hh.swap = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
      hh.nano = magic == 0xa1b23c4du || magic == 0x4d3cb2a1u;
      hh.link = (int)(rd32(b + 20, hh.swap) & 0x0FFFFFFF);
      hh.sec0 = n >= 40 ? rd32(b + 24, hh.swap) : 0u;
      auto parts = index_classic_parallel(b, n, hh, T);
      for (auto& p : parts) lists.push_back(std::move(p.pk));
    } else {
      std::vector<Pkt> pk;
      ok = index_pcap(b, n, &pk, &h->err);
      for (int t = 0; t < T && ok; ++t) {
        const size_t lo = pk.size() * (size_t)t / T, hi = pk.size() * (size_t)(t + 1) / T;
        lists.emplace_back(pk.begin() + lo, pk.begin() + hi);
      }
    }
  } else if (b && b != MAP_FAILED) {
    h->err = "file too short";
  }
  if (ok) {
    std::vector<int64_t> base(lists.size() + 1, 0);
    for (size_t t = 0; t < lists.size(); ++t) base[t + 1] = base[t] + (int64_t)lists[t].size();
    h->packets = base.back();
    std::vector<Rows>& loc = h->parts;
    loc.resize(lists.size());
#pragma omp parallel for num_threads(T) schedule(static, 1)
    for (int t = 0; t < (int)lists.size(); ++t) {
      const std::vector<Pkt>& pk = lists[t];
      for (size_t i = 0; i < pk.size(); ++i) decode(b, pk[i], base[t] + (int64_t)i, &loc[t]);
    }
    std::vector<Frag> frags;
    for (auto& r : loc)
      for (auto& f : r.frags) frags.push_back(std::move(f));
    if (!frags.empty()) {  // serial pass: fragments of one datagram may sit in different chunks
      Rows re;
      reassemble(frags, &re);
      if (!re.ts_ns.empty()) {
        Rows a;
        for (auto& r : loc) append_rows(a, r);
        append_rows(a, re);
        loc.clear();
        loc.push_back(packet_order(a));
      } else {
        loc[0].frag_incomplete += re.frag_incomplete;
      }
    }
    for (auto& r : loc) {
      h->rows += (int64_t)r.ts_ns.size();
      h->name_bytes += (int64_t)r.names.size();
      h->a_bytes += (int64_t)r.as.size();
      h->tcp_partial += r.tcp_partial;
      h->frag_incomplete += r.frag_incomplete;
    }
  }
  if (b && b != MAP_FAILED) munmap((void*)b, n);
  ::close(fd);
  return h;
}

ONI_NATIVE_API int oni_pcap_dns_sizes(void* hp, int64_t* rows, int64_t* name_bytes, int64_t* a_bytes,
                                      int64_t* packets) {
  auto* h = (Handle*)hp;
  *rows = h->rows;
  *name_bytes = h->name_bytes;
  *a_bytes = h->a_bytes;
  *packets = h->packets;
  return h->err.empty() ? 0 : 1;
}

// columns of every part copied straight into the caller's arrays, parts in parallel
ONI_NATIVE_API int oni_pcap_dns_fetch(void* hp, int64_t* ts_ns, int32_t* frame_len, uint32_t* ip_src, uint32_t* ip_dst,
                                      int32_t* qtype, int32_t* qclass, int32_t* rcode, int64_t* name_off,
                                      uint8_t* names, int64_t* a_off, uint8_t* as) {
  auto* h = (Handle*)hp;
  const size_t P = h->parts.size();
  std::vector<int64_t> r0(P + 1, 0), n0(P + 1, 0), b0(P + 1, 0);
  for (size_t p = 0; p < P; ++p) {
    r0[p + 1] = r0[p] + (int64_t)h->parts[p].ts_ns.size();
    n0[p + 1] = n0[p] + (int64_t)h->parts[p].names.size();
    b0[p + 1] = b0[p] + (int64_t)h->parts[p].as.size();
  }
  name_off[0] = 0;
  a_off[0] = 0;
#pragma omp parallel for schedule(static, 1)
  for (size_t p = 0; p < P; ++p) {
    const Rows& a = h->parts[p];
    const size_t n = a.ts_ns.size(), o = (size_t)r0[p];
    if (n) {
      std::memcpy(ts_ns + o, a.ts_ns.data(), n * 8);
      std::memcpy(frame_len + o, a.frame_len.data(), n * 4);
      std::memcpy(ip_src + o, a.ip_src.data(), n * 4);
      std::memcpy(ip_dst + o, a.ip_dst.data(), n * 4);
      std::memcpy(qtype + o, a.qtype.data(), n * 4);
      std::memcpy(qclass + o, a.qclass.data(), n * 4);
      std::memcpy(rcode + o, a.rcode.data(), n * 4);
      for (size_t i = 0; i < n; ++i) {
        name_off[o + i + 1] = a.name_end[i] + n0[p];
        a_off[o + i + 1] = a.a_end[i] + b0[p];
      }
    }
    if (!a.names.empty()) std::memcpy(names + n0[p], a.names.data(), a.names.size());
    if (!a.as.empty()) std::memcpy(as + b0[p], a.as.data(), a.as.size());
  }
  return 0;
}

// decoder counters: [0] TCP messages split across segments (skipped), [1] incomplete IPv4 datagrams
ONI_NATIVE_API int oni_pcap_dns_stats(void* hp, int64_t* out) {
  auto* h = (Handle*)hp;
  out[0] = h->tcp_partial;
  out[1] = h->frag_incomplete;
  return 0;
}

ONI_NATIVE_API void oni_pcap_dns_free(void* hp) { delete (Handle*)hp; }

// ------------------------------------------------------------------------------------------------
// pcap writer (synthetic DNS days): Ethernet/IPv4/UDP/DNS responses with one question and
// optional A answers (name compression pointer back to the question).
// ------------------------------------------------------------------------------------------------
ONI_NATIVE_API int64_t oni_pcap_dns_write(const char* path, int64_t n, const int64_t* ts_ns, const uint32_t* ip_server,
                                          const uint32_t* ip_client, const int64_t* name_off, const uint8_t* names,
                                          const int32_t* qtype, const int32_t* rcode, const int32_t* n_answers,
                                          const uint32_t* answer_ip, int32_t pad_to) {
  FILE* f = std::fopen(path, "wb");
  if (!f) return -1;
  const uint32_t hdr[6] = {0xa1b23c4du, 0x00040002u, 0, 0, 65535, 1};  // ns resolution, v2.4, Ethernet
  std::fwrite(hdr, 4, 6, f);
  std::vector<uint8_t> pkt;
  for (int64_t i = 0; i < n; ++i) {
    pkt.clear();
    auto put16 = [&](uint16_t v) { pkt.push_back(v >> 8); pkt.push_back(v & 255); };
    auto put32 = [&](uint32_t v) { put16(v >> 16); put16(v & 0xFFFF); };
    // Ethernet
    for (int k = 0; k < 12; ++k) pkt.push_back((uint8_t)(k < 6 ? 0x02 : 0x04));
    put16(0x0800);
    const size_t ip0 = pkt.size();
    pkt.push_back(0x45); pkt.push_back(0); put16(0); put16((uint16_t)i); put16(0); pkt.push_back(64); pkt.push_back(17);
    put16(0); put32(ip_server[i]); put32(ip_client[i]);
    const size_t udp0 = pkt.size();
    put16(53); put16((uint16_t)(1024 + (i % 60000))); put16(0); put16(0);
    const size_t dns0 = pkt.size();
    const int na = n_answers ? n_answers[i] : 0;
    put16((uint16_t)i); put16((uint16_t)(0x8180 | (rcode[i] & 0xF))); put16(1); put16((uint16_t)na); put16(0); put16(0);
    // question name
    int64_t a = name_off[i], b = name_off[i + 1];
    while (a < b) {
      int64_t e = a;
      while (e < b && names[e] != '.') ++e;
      const int64_t l = e - a;
      if (l > 0 && l < 64) {
        pkt.push_back((uint8_t)l);
        pkt.insert(pkt.end(), names + a, names + e);
      }
      a = e + 1;
    }
    pkt.push_back(0);
    put16((uint16_t)qtype[i]); put16(1);
    for (int k = 0; k < na; ++k) {
      put16(0xC00C); put16(1); put16(1); put32(300); put16(4); put32(answer_ip ? answer_ip[i] + k : 0);
    }
    while ((int32_t)pkt.size() < pad_to) pkt.push_back(0);
    // lengths
    const uint16_t iplen = (uint16_t)(pkt.size() - ip0), udplen = (uint16_t)(pkt.size() - udp0);
    pkt[ip0 + 2] = iplen >> 8; pkt[ip0 + 3] = iplen & 255;
    pkt[udp0 + 4] = udplen >> 8; pkt[udp0 + 5] = udplen & 255;
    uint32_t sum = 0;
    for (int k = 0; k < 20; k += 2) sum += (pkt[ip0 + k] << 8) | pkt[ip0 + k + 1];
    while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
    const uint16_t ck = (uint16_t)~sum;
    pkt[ip0 + 10] = ck >> 8; pkt[ip0 + 11] = ck & 255;
    (void)dns0;
    const uint32_t rec[4] = {(uint32_t)(ts_ns[i] / 1000000000ll), (uint32_t)(ts_ns[i] % 1000000000ll),
                             (uint32_t)pkt.size(), (uint32_t)pkt.size()};
    std::fwrite(rec, 4, 4, f);
    std::fwrite(pkt.data(), 1, pkt.size(), f);
  }
  std::fclose(f);
  return n;
}
