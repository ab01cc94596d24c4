"""String kernels (K04/K06/K07) + DNS/proxy pipelines on the GPU vs the CPU oracle (bitwise)."""
import numpy as np
import pytest
import torch

from oni355.ops import strings as sops
from oni355.ref import strings_spec as ss
from oni355.store.columnar import StringColumn

pytestmark = pytest.mark.gpu

NAMES = ["www.google.com", "news.bbc.co.uk", "x7f9qkj3h2ab.tunnel.biz.", "", "a", "co.uk", "localhost",
         "58.31.225.10.in-addr.arpa", "MAIL.Intel.COM", "_ldap._tcp.dc._msdcs.corp.intel.com",
         "z" * 60 + "." + "q" * 60 + ".example.de"]


def test_domain_features_bitwise(gpu):
    rng = np.random.default_rng(0)
    extra = ["".join(rng.choice(list("abcdefghijklmnopqrstuvwxyz0123456789-."), rng.integers(1, 80)))
             for _ in range(5000)]
    sc = StringColumn.from_list(NAMES + extra)
    top = ss.HashSet([ss.fnv1a(d.encode()) for d in ["google.com", "bbc.co.uk", "intel.com"]])
    want = ss.domain_features(sc.offsets, sc.chars, top, "intel")
    got = sops.domain_features(torch.from_numpy(sc.offsets).to(gpu), torch.from_numpy(sc.chars).to(gpu), top, "intel")
    assert np.array_equal(got[0].cpu().numpy().view(np.uint64), want[0])
    for g, w in zip(got[1:], want[1:]):
        assert np.array_equal(g.cpu().numpy(), w)


def test_string_features_and_pack_bitwise(gpu):
    rng = np.random.default_rng(1)
    strs = ["".join(chr(c) for c in rng.integers(32, 127, rng.integers(0, 400))) for _ in range(3000)]
    sc = StringColumn.from_list(strs)
    wh, wl, we = ss.string_features(sc.offsets, sc.chars)
    gh, gl, ge = sops.string_features(torch.from_numpy(sc.offsets).to(gpu), torch.from_numpy(sc.chars).to(gpu))
    assert np.array_equal(gh.cpu().numpy().view(np.uint64), wh)
    assert np.array_equal(gl.cpu().numpy(), wl) and np.array_equal(ge.cpu().numpy(), we)
    n = 10_001
    keys = [rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) for _ in range(3)]
    cuts = [np.sort(rng.integers(0, 2**32, m, dtype=np.uint64).astype(np.uint32)) for m in (9, 4, 4)]
    raws = [rng.integers(0, 70000, n).astype(np.int32), rng.integers(0, 16, n).astype(np.int32)]
    top = rng.integers(0, 3, n).astype(np.uint8)
    want = ss.pack_words(keys, cuts, [33, 29, 26], raws, [0xFFFF, 0xF], [4, 0], top, 3, 37)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)  # noqa: E731
    got = sops.pack_words([t(k.view(np.int32)) for k in keys], cuts, [33, 29, 26], [t(r) for r in raws],
                          [0xFFFF, 0xF], [4, 0], raw8=t(top), r8mask=3, r8shift=37)
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)


def test_dns_pipeline_gpu_matches_cpu(gpu):
    from oni355.pipeline.dns import run_dns
    from oni355.synth.dns import generate_dns
    day = generate_dns(20_000, seed=4)
    kw = dict(K=50, sweeps=5, maxresults=100, top_domains=day.top_domains, user_domain="intel")
    rc = run_dns(day.cols, device="cpu", **kw)
    rg = run_dns(day.cols, device=gpu, **kw)
    assert np.array_equal(rc.rows, rg.rows) and np.array_equal(rc.scores, rg.scores)
    assert np.array_equal(rc.words, rg.words)


def test_proxy_pipeline_gpu_matches_cpu(gpu):
    from oni355.pipeline.proxy import run_proxy
    from oni355.synth.proxy import generate_proxy
    day = generate_proxy(10_000, seed=4)
    rc = run_proxy(day.cols, K=20, sweeps=5, maxresults=100, device="cpu", top_domains=["google.com"])
    rg = run_proxy(day.cols, K=20, sweeps=5, maxresults=100, device=gpu, top_domains=["google.com"])
    assert np.array_equal(rc.rows, rg.rows) and np.array_equal(rc.scores, rg.scores)


def test_domain_features_public_suffix_table_bitwise(gpu, tmp_path):
    """The kernel's table-driven registered-domain split == the oracle on adversarial names, with the
    built-in list and with a custom PSL file (deep, wildcard and exception rules)."""
    from oni355.ref import psl
    from oni355.store.columnar import StringColumn
    names = ["a.b.www.ck", "x.y.ck", "ck", "www.ck", "x.city.kawasaki.jp", "a.b.c.d.e.f.g.h.example.co.uk",
             "co.uk", ".", "..", "a..b.com", "", "x", "cdn.foo.github.io", "WWW.BBC.CO.UK.", "q.keep.dyn.example.com",
             "z.x.y.dyn.example.com", "s.school.pvt.k12.ma.us", "evil.co.zz", "-.-.-", "a" * 250 + ".com"]
    p = tmp_path / "psl.dat"
    p.write_text("com\nexample.com\n*.dyn.example.com\n!keep.dyn.example.com\npvt.k12.ma.us\nus\n")
    for rules in (psl.default_rules(), psl.SuffixRules.load(str(p))):
        sc = StringColumn.from_list(names)
        want = ss.domain_features(sc.offsets, sc.chars, None, "", rules)
        got = sops.domain_features(torch.from_numpy(sc.offsets).to(gpu), torch.from_numpy(sc.chars).to(gpu), None, "",
                                   rules)
        for w, g in zip(want, got):
            assert np.array_equal(np.asarray(w).view(np.uint8), g.cpu().numpy().view(np.uint8))


def test_category_codes_match_host_rules(gpu):
    """k_category_codes == proxy.method_code / ctype_class (trim, case fold, longest pattern)."""
    from oni355.pipeline import proxy as px
    meths = ["GET", " get ", "Post", "PUT\t", "head", "CONNECT", "options", "DELETE", "trace", "PATCH", "GETX", "",
             "-", "OTHER", "g e t", "pOsT "]
    ctypes = ["text/html", "TEXT/HTML; charset=utf-8", " text/plain", "image/png", "application/javascript",
              "application/json", "application/octet-stream", "application/x-foo", "video/mp4", "audio/ogg",
              "multipart/form-data", "", "-", " - ", "weird/type", "textual", "application", "IMAGE/"]
    for vals, pats, fold, dflt, fn in ((meths, px.METHOD_PATTERNS, 1, 0, px.method_code),
                                       (ctypes, px.CTYPE_PATTERNS, 2, 10, px.ctype_class)):
        col = StringColumn.from_list(vals * 50)
        off = torch.from_numpy(col.offsets.astype(np.int64)).to(gpu)
        ch = torch.from_numpy(col.chars).to(gpu)
        got = sops.category_codes(off, ch, pats, fold, dflt).cpu().numpy()
        assert got.tolist() == [fn(v) for v in vals * 50]
