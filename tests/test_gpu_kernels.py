"""HIP kernels vs the NumPy specification oracle (bitwise where the spec is exact)."""
import numpy as np
import pytest
import torch

from oni355 import ops
from oni355.models.corpus import build_corpus
from oni355.models.gibbs import GibbsConfig, GibbsLDA
from oni355.ref import spec

pytestmark = pytest.mark.gpu


def _rand_flows(n, seed):
    r = np.random.default_rng(seed)
    return dict(
        hour=r.integers(0, 24, n).astype(np.int32), minute=r.integers(0, 60, n).astype(np.int32),
        second=r.integers(0, 60, n).astype(np.int32),
        ibyt=np.where(r.random(n) < 0.3, 1500, r.integers(0, 10**10, n)).astype(np.int64),
        ipkt=r.integers(0, 5000, n).astype(np.int64),
        sport=np.where(r.random(n) < 0.1, 0, r.integers(0, 65536, n)).astype(np.int32),
        dport=np.where(r.random(n) < 0.1, 0, r.integers(0, 2048, n)).astype(np.int32))


@pytest.mark.parametrize("n", [1, 63, 64, 65, 100_003])
def test_flow_keys_and_words(gpu, n):
    f = _rand_flows(n, n)
    T = {k: torch.from_numpy(v) for k, v in f.items()}
    G = {k: v.to(gpu) for k, v in T.items()}
    kc = ops.flow_keys(T["hour"], T["minute"], T["second"], T["ibyt"], T["ipkt"])
    kg = ops.flow_keys(G["hour"], G["minute"], G["second"], G["ibyt"], G["ipkt"])
    for a, b in zip(kc, kg):
        assert torch.equal(a, b.cpu())
    cuts = [np.sort(np.random.default_rng(1).integers(0, 2**32, m, dtype=np.uint64).astype(np.uint32)) for m in (9, 9, 4)]
    wc = ops.flow_wordify(T["sport"], T["dport"], *kc, *cuts)
    wg = ops.flow_wordify(G["sport"], G["dport"], *kg, *cuts)
    for a, b in zip(wc, wg):
        assert torch.equal(a, b.cpu())


@pytest.mark.parametrize("n", [1, 7, 1000, 1_000_003])
def test_quantile_cuts_exact(gpu, n):
    r = np.random.default_rng(n)
    x = np.concatenate([r.normal(size=n // 2).astype(np.float32), np.full(n - n // 2, 3.25, np.float32)])
    keys = torch.from_numpy(spec.f32_key(x).view(np.int32)).to(gpu)
    for fr in (spec.DECILES, spec.QUINTILES):
        got = ops.quantile_cuts(keys, fr)
        want = spec.quantile_cuts(spec.f32_key(x), fr)
        assert np.array_equal(got, want)


@pytest.mark.parametrize("n", [1, 1000, 1_000_003])
def test_quantile_cuts_multi_equals_single(gpu, n):
    """One read-back per radix pass for all features == per-feature cuts == the NumPy oracle."""
    r = np.random.default_rng(n + 1)
    xs = [r.normal(size=n).astype(np.float32), r.integers(0, 50, n).astype(np.float32),
          np.concatenate([r.exponential(size=n // 3), np.full(n - n // 3, 7.0)]).astype(np.float32)]
    keys = [torch.from_numpy(spec.f32_key(x).view(np.int32)).to(gpu) for x in xs]
    frs = [spec.DECILES, spec.QUINTILES, spec.DECILES]
    got = ops.quantile_cuts_multi(keys, frs)
    for g, k, x, fr in zip(got, keys, xs, frs):
        assert np.array_equal(g, ops.quantile_cuts(k, fr))
        assert np.array_equal(g, spec.quantile_cuts(spec.f32_key(x), fr))
    # the device-only pipeline (k_quantile_pick between passes, no read-back) gives the same cuts
    dev = ops.quantile_cuts_dev(keys, frs).cpu().numpy().view(np.uint32)
    assert np.array_equal(dev, np.concatenate(got))


def _toy_tokens(n_docs, V, seed, heavy=True):
    r = np.random.default_rng(seed)
    lens = r.zipf(1.6, n_docs).clip(1, 3000)
    if heavy:
        lens[0] = 5000  # forces a multi-chunk doc
    tdoc = np.repeat(np.arange(n_docs), lens)
    tword = (r.zipf(1.3, tdoc.size) - 1) % V
    keys = ((np.arange(n_docs, dtype=np.int64) * 2654435761 + seed) % (2**31 - 1)).astype(np.int32)  # distinct
    return torch.from_numpy(tdoc), torch.from_numpy(tword), keys


_SAMPLER_CASES = [(20, "dual"), (20, "delta"), (20, "recount"), (20, "atomic"), (20, "wdelta"),
                  (20, "recount+generic"), (20, "wdelta+generic"), (20, "atomic+generic"), (20, "delta+generic"),
                  (7, "dual"), (7, "wdelta"), (32, "wdelta"), (32, "dual"), (12, "recount"), (4, "wdelta"),
                  (50, "recount"), (50, "wdelta"), (50, "dual"), (50, "delta"), (50, "atomic"),
                  (50, "wdelta+generic"), (40, "dual"), (64, "delta"), (80, "wdelta"), (100, "recount"),
                  (100, "wdelta"), (100, "atomic"), (100, "dual"), (100, "delta"), (100, "wdelta+generic"),
                  (128, "recount"), (200, "atomic"), (200, "wdelta")]


@pytest.mark.parametrize("K,mode", _SAMPLER_CASES)
def test_gibbs_bitwise_vs_oracle(gpu, K, mode):
    """Every sweep kernel (k_gibbs_x1 for K <= 32, k_gibbs_ldsg above, the generic k_gibbs
    fallback -- also what runs where n + α is not exact in f32, e.g. α = 50/7) against the NumPy
    oracle of the collapsed conditional, bit for bit, in every count mode."""
    tdoc, tword, keys = _toy_tokens(300, 400, K)
    G, KP = ops.choose_tiling(K)
    cc = build_corpus(tdoc, tword, 300, 400, torch.from_numpy(keys), G, L=64)
    cg = build_corpus(tdoc.to(gpu), tword.to(gpu), 300, 400, torch.from_numpy(keys).to(gpu), G, L=64)
    assert torch.equal(cc.tok_word, cg.tok_word.cpu())
    assert torch.equal(cc.chunk_doc, cg.chunk_doc.cpu())
    sampler = mode.split("+")[1] if "+" in mode else "dense"
    mg = GibbsLDA(cg, GibbsConfig(K=K, seed=1234, use_graph=False, count_mode=mode.split("+")[0], sampler=sampler))
    exact = K not in (7, 12)  # α = 50/K exact in f32 (and below 2^24 documents) selects the fast kernels
    if sampler == "dense":
        assert mg.qpf == ((3 if G == 1 else 2) if exact else 0), (K, mg.qpf)
    mc = GibbsLDA(cc, GibbsConfig(K=K, seed=1234, use_graph=False, count_mode="atomic", sampler="dense"))
    if mode.startswith("wdelta"):
        assert mg.mode == 4
    mc.initialize()
    mg.initialize()
    assert torch.equal(mc.tok_z, mg.tok_z.cpu())
    assert torch.equal(mc.nwk, mg.nwk.cpu())
    assert torch.equal(mc.q, mg.q.cpu())
    assert torch.equal(mc.qfix, mg.qfix.cpu())
    for _ in range(3):
        mc.sweep(1)
        mg.sweep(1)
        assert torch.equal(mc.tok_z, mg.tok_z.cpu())
        assert torch.equal(mc.ndk_cur, mg.ndk_cur.cpu())
        assert torch.equal(mc.nwk, mg.nwk.cpu())
        assert torch.equal(mc.nk_cur, mg.nk_cur.cpu())
        assert torch.equal(mc.q, mg.q.cpu())
        assert torch.equal(mc.qfix, mg.qfix.cpu())
    # invariants
    T = cg.T
    assert int(mg.nwk[:, :K].sum()) == T == int(mg.ndk_cur[:, :K].sum()) == int(mg.nk_cur[:K].sum())
    assert int(mg.nwk.min()) >= 0 and int(mg.ndk_cur.min()) >= 0


@pytest.mark.parametrize("mode,switch", [("auto", 4), ("auto", 0), ("dual", 0), ("delta", 0), ("wdelta", 0)])
def test_graph_replay_matches_eager(gpu, mode, switch):
    tdoc, tword, keys = _toy_tokens(500, 300, 5)
    c = build_corpus(tdoc.to(gpu), tword.to(gpu), 500, 300, torch.from_numpy(keys).to(gpu), 1, L=128)
    a = GibbsLDA(c, GibbsConfig(K=20, seed=9, use_graph=False, count_mode=mode, auto_switch=switch,
                                auto_threshold=0.99))
    b = GibbsLDA(c, GibbsConfig(K=20, seed=9, use_graph=True, count_mode=mode, auto_switch=switch,
                                auto_threshold=0.99))
    a.initialize()
    a.sweep(9)
    b.initialize()
    b.sweep(2)
    b.sweep(7)
    assert b._graph is not None
    if mode == "auto" and switch == 0:
        assert b._delta_on and a._delta_on
    assert torch.equal(a.tok_z, b.tok_z) and torch.equal(a.nwk, b.nwk) and torch.equal(a.ndk_cur, b.ndk_cur)


@pytest.mark.parametrize("L", [32, 128, 256])
def test_x1_sampler_graph_auto_matches_generic(gpu, L):
    """The one-lane sampler k_gibbs_x1 replays the generic k_gibbs bit for bit through the auto count
    mode's recount → wdelta switch, captured in graphs, at several chunk lengths."""
    tdoc, tword, keys = _toy_tokens(3000, 700, 21)
    c = build_corpus(tdoc.to(gpu), tword.to(gpu), 3000, 700, torch.from_numpy(keys).to(gpu), 1, L=L)
    runs = []
    for sampler in ("generic", "x1"):
        m = GibbsLDA(c, GibbsConfig(K=20, seed=77, count_mode="auto", auto_switch=5, sampler=sampler))
        assert m.qpf == {"generic": 0, "x1": 3}[sampler]
        m.initialize()
        m.sweep(12)
        runs.append(m)
    a, b = runs
    assert a._sweep_mode(a.sweeps_done) == 4 == b._sweep_mode(b.sweeps_done)
    assert torch.equal(a.tok_z, b.tok_z) and torch.equal(a.nwk, b.nwk) and torch.equal(a.ndk_cur, b.ndk_cur)
    assert torch.equal(a.q, b.q)


def test_resume_bitwise(gpu):
    tdoc, tword, keys = _toy_tokens(200, 100, 11)
    c = build_corpus(tdoc.to(gpu), tword.to(gpu), 200, 100, torch.from_numpy(keys).to(gpu), 1, L=64)
    a = GibbsLDA(c, GibbsConfig(K=20, seed=3))
    a.initialize()
    a.sweep(6)
    b = GibbsLDA(c, GibbsConfig(K=20, seed=3))
    b.initialize()
    b.sweep(2)
    z = b.canonical_z().cpu()
    r = GibbsLDA(c, GibbsConfig(K=20, seed=3))
    r.load_canonical_z(z, 2)
    r.sweep(4)
    assert torch.equal(a.canonical_z(), r.canonical_z())
    assert torch.equal(a.nwk, r.nwk)


@pytest.mark.parametrize("KS", [20, 64])
def test_score_and_select(gpu, KS):
    r = np.random.default_rng(KS)
    D, V, n = 1000, 700, 50_001
    th = r.random((D, KS)).astype(np.float32) / KS
    ph = (r.random((V, KS)) ** 8).astype(np.float32)
    d1, d2 = r.integers(0, D, n).astype(np.int32), r.integers(0, D, n).astype(np.int32)
    w1, w2 = r.integers(0, V, n).astype(np.int32), r.integers(0, V, n).astype(np.int32)
    want, s1, s2 = spec.score(th, ph, d1, w1, d2, w2)
    t = lambda a: torch.from_numpy(a).to(gpu)  # noqa: E731
    hist = torch.zeros(2048, dtype=torch.int32, device=gpu)
    got, g1, g2 = ops.score(t(th), t(ph), t(d1), t(w1), t(d2), t(w2), tol=0.5, want_parts=True, hist=hist)
    assert np.array_equal(got.cpu().numpy(), want)
    assert np.array_equal(g1.cpu().numpy(), s1) and np.array_equal(g2.cpu().numpy(), s2)
    b = spec.f32_key(want[want < 0.5]) >> np.uint32(21)
    assert np.array_equal(hist.cpu().numpy(), np.bincount(b, minlength=2048))
    idx, sc = ops.select_below(got, 0.5, 1000, cap=n)
    m = (want < 0.5) & ((spec.f32_key(want) >> np.uint32(21)) <= 1000)
    assert np.array_equal(np.sort(idx.cpu().numpy()), np.nonzero(m)[0])


def test_flow_pipeline_gpu_matches_cpu(gpu):
    from oni355.pipeline.flow import run_flow
    from oni355.synth.flow import generate_flows
    day = generate_flows(20_000, seed=5)
    rc = run_flow(day.cols, K=20, sweeps=6, maxresults=200, device="cpu")
    rg = run_flow(day.cols, K=20, sweeps=6, maxresults=200, device=gpu)
    assert np.array_equal(rc.rows, rg.rows)
    assert np.array_equal(rc.scores, rg.scores)
    # the device log-likelihood sums OCML's lgamma (≤ 2 ulp from libm's) over ~5e5 terms in one
    # fused pass (k_tail_partials): equal to ~1e-10 relative, not bit for bit
    assert rc.stats["loglik"] == pytest.approx(rg.stats["loglik"], rel=1e-8)


@pytest.mark.parametrize("two", [True, False])
def test_pair_plan_score_matches_gather(gpu, two):
    from oni355.pipeline import common
    r = np.random.default_rng(3)
    D, V, n, KS = 900, 600, 200_003, 20
    th = torch.from_numpy((r.random((D, KS)) / KS).astype(np.float32)).to(gpu)
    ph = torch.from_numpy((r.random((V, KS)) ** 6).astype(np.float32)).to(gpu)
    dkeys = torch.arange(D, dtype=torch.int64, device=gpu) * 3 + 1
    vocab = torch.arange(V, dtype=torch.int64, device=gpu) * 5 + 2
    sides = [(dkeys[torch.from_numpy(r.integers(0, D, n)).to(gpu)], vocab[torch.from_numpy(r.integers(0, V, n)).to(gpu)])
             for _ in range(2 if two else 1)]
    plan = common.score_plan(dkeys, vocab, sides, tiles=False)
    h1 = torch.zeros(2048, dtype=torch.int32, device=gpu)
    h2 = torch.zeros(2048, dtype=torch.int32, device=gpu)
    got, g1, g2 = (common.to_event_order(plan, x) for x in common.plan_score(th, ph, plan, 0.3, hist=h1,
                                                                             want_parts=True))
    lk = [(common.lookup(dkeys, a), common.lookup(vocab, b)) for a, b in sides]
    args = [x for p in lk for x in p]
    want, w1, w2 = ops.score(th, ph, *args, tol=0.3, want_parts=True, hist=h2)
    assert torch.equal(got, want) and torch.equal(g1, w1)
    if two:
        assert torch.equal(g2, w2)
    assert torch.equal(h1, h2)


@pytest.mark.parametrize("KS", [20, 52])
def test_tile_score_mfma_bitwise_vs_fma_oracle(gpu, KS):
    """k_tile_score (v_mfma_f32_16x16x4_f32 blocks) == the k-ordered fmaf-chain oracle, bit for bit."""
    from oni355.pipeline import common
    r = np.random.default_rng(KS)
    D, V, n = 700, 500, 60_001
    th = (r.random((D, KS)) / KS).astype(np.float32)
    ph = (r.random((V, KS)) ** 6).astype(np.float32)
    th[:, KS - 2:] = 0  # zero padding columns as theta()/phi() produce
    ph[:, KS - 2:] = 0
    dkeys = torch.arange(D, dtype=torch.int64) * 3 + 1
    vocab = torch.arange(V, dtype=torch.int64) * 5 + 2
    # power-law docs so tiles mix dense heavy rows with single-pair rows
    dsel = torch.from_numpy(np.minimum(r.zipf(1.3, n) - 1, D - 1))
    sides = [(dkeys[dsel], vocab[torch.from_numpy(r.integers(0, V, n))])]
    plan_c = common.score_plan(dkeys, vocab, sides, tiles=True)
    want = common.to_event_order(plan_c, common.plan_score(torch.from_numpy(th), torch.from_numpy(ph), plan_c, 0.3)[0])
    g = lambda x: x.to(gpu)  # noqa: E731
    plan_g = common.score_plan(g(dkeys), g(vocab), [(g(a), g(b)) for a, b in sides], tiles=True)
    t = plan_g.tiles
    ps = ops.tile_score(g(torch.from_numpy(th)), g(torch.from_numpy(ph)), t.item_docs, t.item_words, t.item_p0,
                        t.pair_rc, plan_g.pdoc, plan_g.pword)
    ref = spec.dot_rows_fma(th[plan_g.pdoc.cpu().numpy()], ph[plan_g.pword.cpu().numpy()])
    assert np.array_equal(ps.cpu().numpy(), ref)
    got = common.to_event_order(plan_g, common.plan_score(g(torch.from_numpy(th)), g(torch.from_numpy(ph)), plan_g,
                                                          0.3)[0])
    assert torch.equal(got.cpu(), want)


def test_widen_pair_matches_torch_glue(gpu):
    """k_widen_pair == torch.cat + int64 conversion + u32 mask (the flow day's key glue)."""
    g = torch.Generator().manual_seed(5)
    a = torch.randint(-2**31, 2**31 - 1, (100_003,), dtype=torch.int32, generator=g)
    b = torch.randint(-2**31, 2**31 - 1, (100_003,), dtype=torch.int32, generator=g)
    ref = torch.cat([a, b]).to(torch.int64) & 0xFFFFFFFF
    out = ops.widen_pair(a.to(gpu), b.to(gpu))
    assert out.dtype == torch.int64 and torch.equal(out.cpu(), ref)
    assert torch.equal(ops.widen_pair(a, b), ref)


def test_wdelta_recount_far_words_matches_cpu(gpu):
    """k_wdelta_recount on packed records: rows in the LDS table, rows past its cap and words too far
    from their block's first word for 16 bits (read back from wsorted) all give the CPU deltas."""
    r = np.random.default_rng(3)
    KS = 8
    words = np.sort(r.choice(3_000_000, 900, replace=False)).astype(np.int32)
    ws = torch.from_numpy(np.repeat(words, r.integers(1, 60, words.size)).astype(np.int32))
    T = ws.numel()
    rec = ops.wdelta_records(ws)
    zz = torch.from_numpy(r.integers(0, KS, (T, 2)).astype(np.int32))
    chg = torch.from_numpy(r.random(T) < 0.3)
    low = (zz[:, 0] | zz[:, 1] << 8).to(torch.int16)
    rec.view(torch.int16).view(-1, 2)[:, 0] = torch.where(chg, low, torch.zeros_like(low))
    bits = np.zeros((T + 31) // 32 + 1, dtype=np.uint32)
    pos = np.nonzero(chg.numpy())[0]
    np.bitwise_or.at(bits, pos >> 5, (np.uint32(1) << (pos & 31).astype(np.uint32)))
    V = int(words[-1]) + 1
    out = {}
    for dev in ("cpu", gpu):
        wb = torch.from_numpy(bits.view(np.int32).copy()).to(dev)
        d = torch.zeros(V, KS, dtype=torch.int32, device=dev)
        ops.wdelta_recount(wb, ws.to(dev), rec.to(dev), d, KS)
        assert not bool(wb.any())
        out[dev] = d.cpu()
    assert torch.equal(out["cpu"], out[gpu])
    assert int(out["cpu"].abs().sum()) > 0


@pytest.mark.parametrize("K,force_generic", [(20, False), (20, True), (50, False), (50, True)])
def test_exact_guard_picks_the_row_kernel_per_sweep_bitwise(gpu, monkeypatch, K, force_generic):
    """A document longer than the range in which n + α is exact in f32 (α = 0.5 + 2^-10: counts up
    to 16,381) no longer sends every sweep to the generic kernel: k_exact_guard checks the long rows'
    sweep-start counts on the device and the row kernel (k_gibbs_x1 / k_gibbs_ldsg) or its generic
    twin runs -- the oracle's draws either way. ONI_EXACT_GUARD_LIMIT forces the generic side."""
    from oni355.models import gibbs as gm
    if force_generic:
        monkeypatch.setenv("ONI_EXACT_GUARD_LIMIT", "10")
    r = np.random.default_rng(K)
    D, V = 120, 300
    lens = r.zipf(1.6, D).clip(1, 500)
    lens[0] = 20_000
    tdoc = torch.from_numpy(np.repeat(np.arange(D), lens))
    tword = torch.from_numpy((r.zipf(1.3, int(lens.sum())) - 1) % V)
    keys = torch.from_numpy(((np.arange(D, dtype=np.int64) * 2654435761 + 7) % (2**31 - 1)).astype(np.int32))
    G, _ = ops.choose_tiling(K)
    alpha = 0.5 + 2.0 ** -10
    cc = build_corpus(tdoc, tword, D, V, keys, G, L=64)
    cg = build_corpus(tdoc.to(gpu), tword.to(gpu), D, V, keys.to(gpu), G, L=64)
    assert not gm._alpha_in_row_exact(alpha, cg.max_doc_len())
    mc = GibbsLDA(cc, GibbsConfig(K=K, alpha=alpha, seed=5, use_graph=False, count_mode="atomic", sampler="dense"))
    mg = GibbsLDA(cg, GibbsConfig(K=K, alpha=alpha, seed=5, count_mode="wdelta", sampler="dense"))
    assert mg._guard is not None and mg.qpf == (3 if G == 1 else 2)
    assert mg._guard["rows"].numel() == 1 or force_generic  # only the long document can leave the range
    for m in (mc, mg):
        m.initialize()
    for n in (1, 4, 2):
        mc.sweep(n)
        mg.sweep(n)
        assert int(mg._guard["flag"].item()) == (0 if force_generic else 1)
        for a, b in ((mc.tok_z, mg.tok_z), (mc.nwk, mg.nwk), (mc.ndk_cur, mg.ndk_cur), (mc.q, mg.q)):
            assert torch.equal(a, b.cpu())
    mg.close()
