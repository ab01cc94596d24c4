"""Pure-CPU tests of the behaviour spec: word rules, bins, quantiles, config, file formats."""
import os

import numpy as np
import pytest
import torch

from oni355 import config, ops
from oni355.io import ldac
from oni355.ref import spec


# --- flow port rule: every row of SURVEY.md §2.8 --------------------------------------------------
@pytest.mark.parametrize("sport,dport,port,sdir,ddir", [
    (0, 0, 0, 0, 0),
    (0, 80, 80, 0, 1),          # sport=0, dport>0 -> dport, dst gets -1_
    (443, 0, 443, 1, 0),        # dport=0, sport>0 -> sport, src gets -1_
    (22, 80, spec.PORT_111111, 0, 0),
    (1024, 1024, spec.PORT_111111, 0, 0),
    (80, 51000, 80, 1, 0),      # sport <= 1024 < dport -> sport, src gets -1_
    (51000, 443, 443, 0, 1),    # dport <= 1024 < sport -> dport, dst gets -1_
    (1025, 1025, spec.PORT_333333, 0, 0),
    (6881, 51413, spec.PORT_333333, 0, 0),
])
def test_port_rule_table(sport, dport, port, sdir, ddir):
    p, s, d = spec.flow_port_rule(np.array([sport]), np.array([dport]))
    assert (p[0], s[0], d[0]) == (port, sdir, ddir)


def test_word_render_roundtrip():
    words = spec.flow_wordify(np.array([80, 0, 6000, 22]), np.array([51000, 0, 7000, 25]),
                              spec.f32_key(np.array([1.0, 2.0, 3.0, 23.9], np.float32)),
                              np.array([10, 20, 30, 10**9], np.uint32), np.array([1, 2, 3, 4], np.uint32),
                              spec.f32_key(np.arange(9, dtype=np.float32) * 2.5),
                              np.array([5, 15, 25, 35, 45, 55, 65, 75, 85], np.uint32),
                              np.array([1, 2, 3, 4], np.uint32))
    strs = [spec.flow_word_str(int(w)) for w in np.concatenate(words)]
    assert strs[0] == "-1_80_1_1_0"  # src of (80 -> 51000): -1_ prefix
    assert strs[4] == "80_1_1_0"
    assert strs[1] == "0_1_2_1" and strs[5] == "0_1_2_1"
    assert strs[2].startswith("333333_") and strs[3].startswith("111111_")
    for w, s in zip(np.concatenate(words), strs):
        assert spec.flow_word_from_str(s) == int(w)


def test_bin_semantics():
    cuts = np.array([10, 20, 30], np.uint32)
    assert list(spec.bin_keys(np.array([0, 10, 11, 20, 21, 30, 31], np.uint32), cuts)) == [0, 0, 1, 1, 2, 2, 3]


@pytest.mark.parametrize("n", [1, 2, 9, 10, 11, 1001])
def test_quantile_ranks_and_cuts(n):
    x = np.random.default_rng(n).permutation(n).astype(np.uint32)
    cuts = spec.quantile_cuts(x, spec.DECILES)
    s = np.sort(x)
    for (num, den), c in zip(spec.DECILES, cuts):
        r = -(-num * n // den) - 1
        assert c == s[max(r, 0)]
    # radix-select path (used on device and for DP) agrees with the sort path
    k = torch.from_numpy(x.view(np.int32))
    assert np.array_equal(ops.quantile_cuts(k, spec.DECILES, allreduce=lambda h: h), cuts)


def test_f32_key_order():
    x = np.array([-np.inf, -3.5, -0.0, 0.0, 1e-30, 2.0, np.inf], np.float32)
    k = spec.f32_key(x)
    assert np.all(np.diff(k.astype(np.int64)) >= 0)
    assert np.array_equal(spec.key_f32(k), x)


def test_philox_known_answer():
    # Random123 Philox4x32-10 known-answer vector (counter 0, key 0)
    r = spec.philox10(0, 0, 0, 0, 0, 0)
    assert [int(v) for v in r] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]


# --- config ------------------------------------------------------------------------------------------
def test_duxbay_parsing(tmp_path):
    p = tmp_path / "duxbay.conf"
    p.write_text('# comment\nUSER_DOMAIN="intel"\nTOPIC_COUNT=50\nLUSER=/home/oni\nLPATH=${LUSER}/ml\n'
                 "DUPFACTOR=500\nTOL=1e-6\nMAXRESULTS=1000\nNODES=(node1 node2)\n")
    cfg = config.load_config(str(p), env={"ONI_SWEEPS": "33"}, MAXRESULTS=77)
    assert cfg.USER_DOMAIN == "intel" and cfg.TOPIC_COUNT == 50 and cfg.DUPFACTOR == 500
    assert cfg.LPATH == "/home/oni/ml" and cfg.TOL == 1e-6 and cfg.SWEEPS == 33 and cfg.MAXRESULTS == 77
    assert cfg.extra["LUSER"] == "/home/oni"


def test_lda_settings():
    s = config.parse_lda_settings("var max iter 20\nvar convergence 1e-6\nem max iter 150\nem convergence 1e-4\n"
                                  "alpha fixed\nsweeps 300\nbeta 0.05\n")
    assert s["em_max_iter"] == 150 and not s["estimate_alpha"] and s["sweeps"] == 300 and s["beta"] == 0.05


# --- lda-c formats -------------------------------------------------------------------------------
def test_ldac_roundtrip(tmp_path):
    pd = np.array([0, 0, 1, 2, 2, 2])
    pw = np.array([3, 7, 1, 0, 5, 9])
    pc = np.array([2, 1, 4, 1, 1, 3])
    f = tmp_path / "model.dat"
    ldac.write_corpus(str(f), pd, pw, pc, 4)
    docs = ldac.read_corpus(str(f))
    assert len(docs) == 4 and list(docs[0][0]) == [3, 7] and list(docs[2][1]) == [1, 1, 3] and docs[3][0].size == 0
    lb = np.log(np.random.default_rng(0).dirichlet(np.ones(10), 3))
    g = np.random.default_rng(1).random((4, 3))
    ldac.write_model(str(tmp_path), "final", lb, g, 0.7)
    assert np.allclose(ldac.read_matrix(str(tmp_path / "final.beta")), lb, atol=1e-9)
    assert ldac.read_other(str(tmp_path / "final.other")) == {"num_topics": 3, "num_terms": 10, "alpha": 0.7}


def test_vem_recovers_topics():
    from oni355.models import vem
    r = np.random.default_rng(0)
    V, K = 60, 3
    phi = np.zeros((K, V))
    for k in range(K):
        phi[k, k * 20:(k + 1) * 20] = 1 / 20
    ptr, ws, cs = [0], [], []
    for d in range(150):
        k = d % K
        w = r.choice(V, 40, p=phi[k])
        u, c = np.unique(w, return_counts=True)
        ws += list(u)
        cs += list(c)
        ptr.append(len(ws))
    res = vem.estimate(np.array(ptr), np.array(ws), np.array(cs), V, K, alpha=0.5, em_max_iter=50, threads=2)
    th = res.theta()
    # every document is (nearly) pure in one topic and documents of one true class share it
    top = th.argmax(1)
    for k in range(K):
        assert len(set(top[k::K])) == 1
    assert th.max(1).mean() > 0.9
    assert np.all(np.diff(res.likelihood[1:]) > -1e-6 * np.abs(res.likelihood[1:-1]).max())


def test_lda_cli(tmp_path):
    import subprocess

    from oni355.ops import native
    ldac.write_corpus(str(tmp_path / "model.dat"), np.repeat(np.arange(30), 2), np.tile([0, 1], 30) + np.repeat(np.arange(30) % 2 * 2, 2),
                      np.full(60, 3), 30)
    (tmp_path / "settings.txt").write_text("var max iter 10\nvar convergence 1e-5\nem max iter 20\nem convergence 1e-4\nalpha estimate\n")
    out = tmp_path / "out"
    subprocess.run([native.binary("lda"), "est", "2.5", "2", str(tmp_path / "settings.txt"), "2",
                    str(tmp_path / "model.dat"), "seeded", str(out)], check=True, capture_output=True)
    assert (out / "final.beta").exists() and (out / "final.gamma").exists() and (out / "word-assignments.dat").exists()
    subprocess.run([native.binary("lda"), "inf", str(tmp_path / "settings.txt"), str(out / "final"),
                    str(tmp_path / "model.dat"), str(tmp_path / "inf")], check=True, capture_output=True)
    g = ldac.read_matrix(str(tmp_path / "inf-gamma.dat"))
    assert g.shape == (30, 2)
    assert os.path.exists(str(tmp_path / "inf-lda-lhood.dat"))


def test_fma_f32_matches_exact_rounding():
    from fractions import Fraction
    r = np.random.default_rng(3)
    n = 3000
    a = (r.random(n) * 100).astype(np.float32)
    b = (r.random(n) * 1e-3).astype(np.float32)
    c = r.random(n).astype(np.float32)
    # midpoint cases: c + a*b lands exactly on / next to a half-ulp of c
    a[:1000] = np.float32(1.0) + np.float32(2.0 ** -23) * r.integers(0, 4, 1000).astype(np.float32)
    b[:1000] = np.float32(2.0 ** -24)
    c[:1000] = np.float32(1.0)
    got = spec.fma_f32(a, b, c)
    for i in range(n):
        v = Fraction(float(a[i])) * Fraction(float(b[i])) + Fraction(float(c[i]))
        f = np.float32(float(v))
        cands = [np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))]
        best = min(cands, key=lambda x: (abs(Fraction(float(x)) - v), int(np.float32(x).view(np.uint32)) & 1))
        assert got[i] == best, i


def test_lds_sampler_oracle_keeps_counts_consistent():
    import torch

    from oni355.models.corpus import build_corpus
    from oni355.models.gibbs import GibbsConfig, GibbsLDA
    r = np.random.default_rng(4)
    lens = r.integers(1, 300, 80)
    tdoc = torch.from_numpy(np.repeat(np.arange(80), lens))
    tword = torch.from_numpy(r.integers(0, 50, int(lens.sum())))
    keys = torch.arange(80, dtype=torch.int32) * 7 + 1
    c = build_corpus(tdoc, tword, 80, 50, keys, 1, L=64)
    m = GibbsLDA(c, GibbsConfig(K=20, seed=5, sampler="x1"))
    assert m.qpf == 3
    m.initialize()
    m.sweep(3)
    T = c.T
    assert int(m.nwk[:, :20].sum()) == T == int(m.ndk_cur[:, :20].sum()) == int(m.nk_cur[:20].sum())


def test_auto_count_mode_matches_recount():
    import torch

    from oni355.models.corpus import build_corpus
    from oni355.models.gibbs import GibbsConfig, GibbsLDA
    r = np.random.default_rng(8)
    lens = r.integers(1, 200, 60)
    tdoc = torch.from_numpy(np.repeat(np.arange(60), lens))
    tword = torch.from_numpy(r.integers(0, 40, int(lens.sum())))
    keys = torch.arange(60, dtype=torch.int32) * 11 + 3
    c = build_corpus(tdoc, tword, 60, 40, keys, 1, L=64)
    a = GibbsLDA(c, GibbsConfig(K=20, seed=2, count_mode="auto", auto_switch=3))
    b = GibbsLDA(c, GibbsConfig(K=20, seed=2, count_mode="recount"))
    for m in (a, b):
        m.initialize()
        m.sweep(6)
    assert torch.equal(a.tok_z, b.tok_z) and torch.equal(a.nwk, b.nwk) and torch.equal(a.ndk_cur, b.ndk_cur)


def test_adaptive_auto_mode_switches_and_matches_recount():
    import torch

    from oni355.models.corpus import build_corpus
    from oni355.models.gibbs import GibbsConfig, GibbsLDA
    r = np.random.default_rng(9)
    lens = r.integers(1, 200, 60)
    tdoc = torch.from_numpy(np.repeat(np.arange(60), lens))
    tword = torch.from_numpy(r.integers(0, 40, int(lens.sum())))
    c = build_corpus(tdoc, tword, 60, 40, torch.arange(60, dtype=torch.int32) * 5 + 1, 1, L=64)
    a = GibbsLDA(c, GibbsConfig(K=20, seed=4, count_mode="auto", auto_threshold=0.99))
    b = GibbsLDA(c, GibbsConfig(K=20, seed=4, count_mode="recount"))
    for m in (a, b):
        m.initialize()
        m.sweep(8)
    assert a._delta_on and a.change_log and 0 < a.change_log[0][1] < 1
    assert torch.equal(a.tok_z, b.tok_z) and torch.equal(a.nwk, b.nwk) and torch.equal(a.nk_cur, b.nk_cur)


def test_wdelta_count_mode_matches_recount():
    """Word-bitmap delta bookkeeping (MODE 4) reproduces the full recount's chain exactly."""
    import torch

    from oni355.models.corpus import build_corpus
    from oni355.models.gibbs import GibbsConfig, GibbsLDA
    r = np.random.default_rng(10)
    lens = r.integers(1, 300, 50)
    tdoc = torch.from_numpy(np.repeat(np.arange(50), lens))
    tword = torch.from_numpy(r.integers(0, 60, int(lens.sum())))
    c = build_corpus(tdoc, tword, 50, 60, torch.arange(50, dtype=torch.int32) * 7 + 2, 1, L=64)
    a = GibbsLDA(c, GibbsConfig(K=20, seed=6, count_mode="wdelta"))
    b = GibbsLDA(c, GibbsConfig(K=20, seed=6, count_mode="recount"))
    for m in (a, b):
        m.initialize()
        m.sweep(5)
    assert torch.equal(a.tok_z, b.tok_z) and torch.equal(a.nwk, b.nwk) and torch.equal(a.nk_cur, b.nk_cur)
    assert not bool(a.wbits.any())  # the recount clears every bit it consumed
    rec = a.zz_w.view(torch.int16).view(-1, 2)[:, 1].to(torch.int32) & 0xFFFF
    ws = c.wsorted.to(torch.int32)
    assert torch.equal(rec[:c.T], ws - ws[0])  # one 8192-position block: rows below its first word


def test_wdelta_records_rows_and_far_words():
    """The MODE-4 record array holds each position's word row in its 8192-position recount block,
    0xFFFF when the gap does not fit 16 bits, and zero topic halves."""
    import torch

    from oni355 import ops
    ws = torch.tensor([3] * 5000 + [70000] * 3192 + [70001] * 10 + [200000] * 5, dtype=torch.int32)
    rec = ops.wdelta_records(ws)
    assert rec.dtype == torch.int32 and rec.numel() == ws.numel()
    halves = rec.view(torch.int16).view(-1, 2).to(torch.int32) & 0xFFFF
    assert int(halves[:, 0].abs().sum()) == 0
    hi = halves[:, 1]
    assert hi[:5000].eq(0).all() and hi[5000:8192].eq(0xFFFF).all()  # 69997 > 0xFFFF: read wsorted
    assert hi[8192:8202].eq(0).all() and hi[8202:].eq(0xFFFF).all()  # next block starts at 70001


def test_auto_with_dual_early_sweeps_matches_recount(monkeypatch):
    """ONI_AUTO_EARLY=dual (word-sorted z copy kept current in the early sweeps, streamed recount)
    leaves the chain bitwise equal to the plain recount mode."""
    import torch

    from oni355.models.corpus import build_corpus
    from oni355.models.gibbs import GibbsConfig, GibbsLDA

    monkeypatch.setenv("ONI_AUTO_EARLY", "dual")
    r = np.random.default_rng(8)
    lens = r.integers(1, 200, 60)
    tdoc = torch.from_numpy(np.repeat(np.arange(60), lens))
    tword = torch.from_numpy(r.integers(0, 40, int(lens.sum())))
    keys = torch.arange(60, dtype=torch.int32) * 11 + 3
    c = build_corpus(tdoc, tword, 60, 40, keys, 1, L=64)
    a = GibbsLDA(c, GibbsConfig(K=20, seed=5, count_mode="auto", auto_switch=4))
    assert a.early == 3
    b = GibbsLDA(c, GibbsConfig(K=20, seed=5, count_mode="recount"))
    for m in (a, b):
        m.initialize()
        m.sweep(9)
    assert torch.equal(a.tok_z, b.tok_z) and torch.equal(a.nwk, b.nwk) and torch.equal(a.ndk_cur, b.ndk_cur)


def test_tiling_choice_and_alpha_in_row_rule(monkeypatch):
    """Unit widths: 1 lane to K = 32, 2 lanes to 56, 4 lanes to 112 (wide, default), the old
    4/8/16-lane units with ONI_TILING=narrow; KS = G·KP covers K with KP a multiple of 4. The
    n + α LDS rows are allowed only where every n + α is exact in f32."""
    from oni355 import ops
    from oni355.models.gibbs import _alpha_in_row_exact

    for K in range(1, 256):
        G, KP = ops.choose_tiling(K)
        assert G * KP >= K and KP % 4 == 0 and G in (1, 2, 4, 8, 16)
    assert ops.choose_tiling(20) == (1, 20) and ops.choose_tiling(50) == (2, 28)
    assert ops.choose_tiling(100) == (4, 28) and ops.choose_tiling(120) == (8, 16)
    monkeypatch.setenv("ONI_TILING", "narrow")
    assert ops.choose_tiling(50) == (4, 16) and ops.choose_tiling(100) == (8, 16)
    assert _alpha_in_row_exact(2.5, 10**6) and _alpha_in_row_exact(0.5, (1 << 22))
    assert not _alpha_in_row_exact(0.5, 1 << 23)  # 2^23 + 0.5 needs 25 significant bits
    assert not _alpha_in_row_exact(0.1, 10) and not _alpha_in_row_exact(50 / 7, 10)


def test_x01_pack_policy(monkeypatch):
    """ONI_X01_PACK: "1" always, "0" never, "auto" only for Δ buffers of at least
    ONI_X01_PACK_MIN_BYTES (default 4 MiB: the flow day's 0.46 MB buffer stays unpacked)."""
    import torch

    from oni355.models import gibbs as gm
    from oni355.models.corpus import build_corpus

    r = np.random.default_rng(3)
    c = build_corpus(torch.from_numpy(r.integers(0, 20, 500)), torch.from_numpy(r.integers(0, 300, 500)),
                     20, 300, torch.arange(20, dtype=torch.int32), 1, L=64)
    m = gm.GibbsLDA(c, gm.GibbsConfig(K=20, seed=1))
    nbytes = m.dn[0].numel() * 4
    assert nbytes < gm.X01_PACK_MIN_BYTES
    monkeypatch.delenv("ONI_X01_PACK", raising=False)
    assert not m._x01_wanted()
    monkeypatch.setenv("ONI_X01_PACK_MIN_BYTES", str(nbytes))
    assert m._x01_wanted()
    monkeypatch.setenv("ONI_X01_PACK", "0")
    assert not m._x01_wanted()
    monkeypatch.setenv("ONI_X01_PACK", "1")
    monkeypatch.setenv("ONI_X01_PACK_MIN_BYTES", str(1 << 40))
    assert m._x01_wanted()


def test_auto_mode_stops_polling_far_above_threshold():
    """A chain still far above the switch point after POLL_GIVE_UP_SWEEP sweeps stops reading back
    change counts; the chain itself is the recount chain bit for bit."""
    import torch

    from oni355.models import gibbs as gm
    from oni355.models.corpus import build_corpus
    r = np.random.default_rng(12)
    lens = r.integers(1, 120, 40)
    tdoc = torch.from_numpy(np.repeat(np.arange(40), lens))
    tword = torch.from_numpy(r.integers(0, 50, int(lens.sum())))
    c = build_corpus(tdoc, tword, 40, 50, torch.arange(40, dtype=torch.int32) * 5 + 1, 1, L=64)
    a = gm.GibbsLDA(c, gm.GibbsConfig(K=20, seed=3, count_mode="auto", auto_threshold=1e-4))
    b = gm.GibbsLDA(c, gm.GibbsConfig(K=20, seed=3, count_mode="recount"))
    for m in (a, b):
        m.initialize()
        m.sweep(gm.POLL_GIVE_UP_SWEEP + 10)
    assert a._poll_off and not a._delta_on
    assert max(sw for sw, _ in a.change_log) < gm.POLL_GIVE_UP_SWEEP + 4
    assert torch.equal(a.tok_z, b.tok_z) and torch.equal(a.nwk, b.nwk)
