"""DNS/proxy featurization spec (CPU): domain split by the public-suffix table, entropy, top-1M set, pcap."""
import math

import numpy as np
import pytest

from oni355.ref import strings_spec as ss
from oni355.store.columnar import StringColumn


@pytest.mark.parametrize("name,reg,sub,periods", [
    ("www.google.com", "google.com", "www", 2),
    ("google.com", "google.com", "", 1),
    ("news.bbc.co.uk", "bbc.co.uk", "news", 3),
    ("bbc.co.uk", "bbc.co.uk", "", 2),
    ("a.b.c.example.de", "example.de", "a.b.c", 4),
    ("www.spiegel.de.", "spiegel.de", "www", 2),      # trailing root dot
    ("localhost", "localhost", "", 0),
    ("58.31.225.10.in-addr.arpa", "in-addr.arpa", "58.31.225.10", 5),
    ("co.uk", "co.uk", "", 1),
    ("x.amazon.co.jp", "amazon.co.jp", "x", 3),
    # table-driven public suffixes (oni355/data/public_suffix_list.dat): wildcard / exception / private rules
    ("a.b.www.ck", "www.ck", "a.b", 3),                # !www.ck exception under *.ck
    ("x.y.ck", "x.y.ck", "", 2),                       # *.ck wildcard: y.ck is a public suffix
    ("x.city.kawasaki.jp", "city.kawasaki.jp", "x", 3),
    ("cdn.foo.github.io", "foo.github.io", "cdn", 3),  # private-section rule
    ("evil.co.zz", "co.zz", "evil", 2),                # unknown TLD: the implicit "*" rule
    ("WWW.BBC.CO.UK", "BBC.CO.UK", "WWW", 3),          # case-insensitive
])
def test_split_domain(name, reg, sub, periods):
    b = name.encode()
    r, e, p = ss.split_domain(b)
    assert b[r:e].decode() == reg
    assert (b[: r - 1].decode() if r > 0 else "") == sub
    assert p == periods


def test_entropy_matches_formula():
    for s in ["", "a", "aaaa", "abcd", "x7f9qkj3h2", "www"]:
        b = s.encode()
        if not b:
            assert ss.entropy(b) == 0
            continue
        _, c = np.unique(list(b), return_counts=True)
        p = c / c.sum()
        assert float(ss.entropy(b)) == pytest.approx(-(p * np.log2(p)).sum(), abs=2e-6)


def test_hash_set():
    hs = ss.HashSet([ss.fnv1a(d.encode()) for d in ["google.com", "bbc.co.uk", "intel.com"]])
    assert ss.fnv1a(b"GOOGLE.com") in hs and ss.fnv1a(b"bbc.co.uk") in hs and ss.fnv1a(b"evil.biz") not in hs


def test_domain_features_top_and_user():
    names = ["www.google.com", "mail.intel.com", "x.y.evil.biz", "intel.com"]
    sc = StringColumn.from_list(names)
    top = ss.HashSet([ss.fnv1a(b"google.com")])
    rh, t, sl, en, per = ss.domain_features(sc.offsets, sc.chars, top, "intel")
    assert list(t) == [1, 2, 0, 2]
    assert list(sl) == [3, 4, 3, 0]
    assert list(per) == [2, 2, 3, 1]
    assert en[2] == pytest.approx(1.0 + 0.0 * math.log2(1), abs=1e-6) or en[2] > 0


def test_pack_words_layout():
    from oni355.pipeline.dns import word_str
    keys = [np.array([5, 50], np.uint32), np.array([1, 2], np.uint32)]
    w = ss.pack_words(keys, [[10, 20], [1]], [33, 29], [np.array([16, 1]), np.array([3, 0])], [0xFFFF, 0xF], [4, 0],
                      np.array([2, 0], np.uint8), 3, 37)
    assert int(w[0]) == (2 << 37) | (0 << 33) | (0 << 29) | (16 << 4) | 3
    assert int(w[1]) == (2 << 33) | (1 << 29) | (1 << 4)
    assert word_str(int(w[0])).startswith("2_0_0_")


def test_pcap_roundtrip(tmp_path):
    from oni355.io.decoders import read_pcap_dns
    from oni355.synth.dns import generate_dns, write_pcap
    day = generate_dns(3000, seed=8)
    write_pcap(day, str(tmp_path / "x.pcap"))
    d = read_pcap_dns(str(tmp_path / "x.pcap"))
    assert d["_packets"] == 3000
    for k in ("unix_tstamp", "frame_len", "ip_src", "ip_dst", "dns_qry_type", "dns_qry_class", "dns_qry_rcode"):
        assert np.array_equal(np.asarray(d[k]), np.asarray(day.cols[k])), k
    assert d["dns_qry_name"].to_list() == day.cols["dns_qry_name"].to_list()
    assert d["dns_a"].to_list() == day.cols["dns_a"].to_list()


def test_pcap_truncated_and_garbage(tmp_path):
    from oni355.io.decoders import read_pcap_dns
    from oni355.synth.dns import generate_dns, write_pcap
    day = generate_dns(200, seed=1)
    p = tmp_path / "t.pcap"
    write_pcap(day, str(p))
    raw = p.read_bytes()
    (tmp_path / "cut.pcap").write_bytes(raw[: len(raw) // 2 + 7])
    d = read_pcap_dns(str(tmp_path / "cut.pcap"))
    assert 0 < len(d["dns_qry_name"]) < 200
    (tmp_path / "bad.pcap").write_bytes(b"\x00" * 100)
    with pytest.raises(OSError):
        read_pcap_dns(str(tmp_path / "bad.pcap"))


def test_custom_suffix_list_drives_the_split(tmp_path):
    """A PSL file (Mozilla format) replaces the built-in rules: deep, wildcard and exception rules."""
    from oni355.ref import psl
    p = tmp_path / "psl.dat"
    p.write_text("// test list\ncom\nexample.com\n*.dyn.example.com\n!keep.dyn.example.com\npvt.k12.ma.us\nus\n")
    rules = psl.SuffixRules.load(str(p))
    cases = {b"a.b.example.com": b"b.example.com", b"x.y.dyn.example.com": b"x.y.dyn.example.com",
             b"z.x.y.dyn.example.com": b"x.y.dyn.example.com", b"q.keep.dyn.example.com": b"keep.dyn.example.com",
             b"s.school.pvt.k12.ma.us": b"school.pvt.k12.ma.us", b"www.google.com": b"google.com"}
    for name, reg in cases.items():
        r, e, _ = ss.split_domain(name, rules)
        assert name[r:e] == reg, (name, name[r:e])
    # the built-in list still splits co.uk names; the custom one does not know .uk rules
    r, e, _ = ss.split_domain(b"news.bbc.co.uk", rules)
    assert b"news.bbc.co.uk"[r:e] == b"co.uk"
