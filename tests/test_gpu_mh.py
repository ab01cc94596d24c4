"""k_mh_alias / k_gibbs_mh / k_gibbs_mh_init (csrc/kernels/gibbs_mh.hip) against their NumPy oracle
(spec.mh_tables, spec.gibbs_pass_mh, spec.gibbs_pass init), bit for bit, in every count mode,
with one and two doc moves, one-chunk and multi-chunk documents, eager and graph-captured."""
import numpy as np
import pytest
import torch

from oni355 import ops
from oni355.models.corpus import build_corpus
from oni355.models.gibbs import GibbsConfig, GibbsLDA
from oni355.ref import spec

pytestmark = pytest.mark.gpu


def _toy(n_docs, V, seed):
    r = np.random.default_rng(seed)
    lens = r.zipf(1.6, n_docs).clip(1, 3000)
    lens[0] = 5000  # a heavy doc: many chunks, several waves
    tdoc = np.repeat(np.arange(n_docs), lens)
    tword = (r.zipf(1.3, tdoc.size) - 1) % V
    keys = ((np.arange(n_docs, dtype=np.int64) * 2654435761 + seed) % (2**31 - 1)).astype(np.int32)
    return torch.from_numpy(tdoc), torch.from_numpy(tword), keys


@pytest.mark.parametrize("K,V", [(7, 1000), (40, 1000), (100, 1000), (255, 1000), (40, 70001)])
def test_alias_tables_bitwise(gpu, K, V):
    """Word proposal tables -- alias records (k_mh_alias; V ≥ 65536: rows go out one at a time,
    lanes along k) and CDF rows (k_mh_cdf: buckets of 8 topics up to K = 128, 16 above) -- and the
    multi-chunk documents' alias rows, bit for bit."""
    r = np.random.default_rng(K)
    KS = (K + 3) // 4 * 4
    q = np.zeros((V, KS), np.float32)
    q[:, :K] = (r.random((V, K)) ** 6 * 0.3 + 1e-6).astype(np.float32)
    q[3, :K] = 0.01  # a flat row
    ndk = r.integers(0, 50, (200, KS)).astype(np.int32) * (r.random((200, KS)) < 0.2)
    ndk[:, K:] = 0
    rows = np.array([0, 5, 7, 199], np.int32)
    nk = r.integers(0, 10**6, KS).astype(np.int32)
    dev = torch.device(gpu)
    args = [torch.from_numpy(x).to(dev) for x in (q, nk, ndk, rows)]
    for word in ("alias", "cdf"):
        wt, ws, da, g = spec.mh_tables(q, nk, ndk, rows, K, 0.37, 17.5, word=word)
        out = [torch.zeros(len(rows), K, dtype=torch.int32, device=dev), torch.zeros(KS, device=dev)]
        if word == "cdf":
            tabs = dict(wcdf=torch.zeros(V, 16, device=dev))
        else:
            tabs = dict(walias=torch.zeros(V, K, 4, dtype=torch.int32, device=dev), wsum=torch.zeros(V, device=dev))
        ops.mh_tables(*args[:2], args[2], args[3], K, 0.37, 17.5, *out, **tabs)
        if word == "cdf":
            assert np.array_equal(tabs["wcdf"].cpu().numpy(), wt)
        else:
            assert np.array_equal(tabs["walias"].cpu().numpy().view(np.uint32), wt)
            assert np.array_equal(tabs["wsum"].cpu().numpy(), ws)
        assert np.array_equal(out[0].cpu().numpy().view(np.uint32), da)
        assert np.array_equal(out[1].cpu().numpy(), g)


_CASES = [(100, "recount", 1, 64), (100, "wdelta", 1, 64), (100, "atomic", 1, 64), (100, "dual", 1, 64),
          (100, "delta", 1, 64), (100, "recount", 2, 64), (100, "wdelta", 2, 32), (40, "wdelta", 1, 32),
          (7, "recount", 1, 64), (255, "wdelta", 2, 64), (64, "dual", 2, 127), (100, "wdelta", 3, 64),
          (100, "recount", 4, 127), (40, "dual", 4, 32)]


@pytest.mark.parametrize("word", ["alias", "cdf"])
@pytest.mark.parametrize("K,mode,dm,L", _CASES)
def test_mh_sweep_bitwise_vs_oracle(gpu, K, mode, dm, L, word, monkeypatch):
    monkeypatch.setenv("ONI_MH_DOC_MOVES", str(dm))
    monkeypatch.setenv("ONI_MH_WORD", word)
    tdoc, tword, keys = _toy(300, 400, K + dm)
    G, KP = ops.choose_tiling(K, "mh")
    cc = build_corpus(tdoc, tword, 300, 400, torch.from_numpy(keys), G, L=L)
    cg = build_corpus(tdoc.to(gpu), tword.to(gpu), 300, 400, torch.from_numpy(keys).to(gpu), G, L=L)
    assert torch.equal(cc.chunk_doc, cg.chunk_doc.cpu())
    mc = GibbsLDA(cc, GibbsConfig(K=K, seed=4321, use_graph=False, count_mode="atomic", sampler="mh"))
    mg = GibbsLDA(cg, GibbsConfig(K=K, seed=4321, use_graph=False, count_mode=mode, sampler="mh"))
    assert mg.qpf == ops.SAMPLER_MH and mg.mh_doc_moves == dm and mg.mh_word == mc.mh_word == word
    mc.initialize()
    mg.initialize()
    assert torch.equal(mc.tok_z, mg.tok_z.cpu())
    assert torch.equal(mc.ndk_cur, mg.ndk_cur.cpu())
    assert torch.equal(mc.nwk, mg.nwk.cpu())
    for _ in range(3):
        mc.sweep(1)
        mg.sweep(1)
        if mg.mh_word == "cdf":
            assert torch.equal(mc.wcdf, mg.wcdf.cpu())
        else:
            assert torch.equal(mc.walias, mg.walias.cpu()) and torch.equal(mc.wsum, mg.wsum.cpu())
        assert torch.equal(mc.dalias, mg.dalias.cpu()) and torch.equal(mc.mh_g, mg.mh_g.cpu())
        assert torch.equal(mc.tok_z, mg.tok_z.cpu())
        assert torch.equal(mc.ndk_cur, mg.ndk_cur.cpu())
        assert torch.equal(mc.nwk, mg.nwk.cpu())
        assert torch.equal(mc.nk_cur, mg.nk_cur.cpu())
    T = cg.T
    assert int(mg.nwk[:, :K].sum()) == T == int(mg.ndk_cur[:, :K].sum()) == int(mg.nk_cur[:K].sum())
    assert int(mg.nwk.min()) >= 0 and int(mg.ndk_cur.min()) >= 0


@pytest.mark.parametrize("mode", ["recount", "wdelta"])
def test_mh_round5_gathers_match_the_oracle(gpu, mode, monkeypatch):
    """ONI_SAMPLER_AB=32 (k_gibbs_mh's round-5 level-1 CDF gathers, kept for A/B) draws the same
    chain as the oracle, like the default cooperative gathers."""
    monkeypatch.setenv("ONI_SAMPLER_AB", "32")
    test_mh_sweep_bitwise_vs_oracle(gpu, 100, mode, 2, 64, "cdf", monkeypatch)


def test_mh_graph_auto_matches_eager(gpu):
    """Graph-captured sweeps (the auto count mode's recount → wdelta switch) equal eager ones."""
    tdoc, tword, keys = _toy(2000, 700, 3)
    c = build_corpus(tdoc.to(gpu), tword.to(gpu), 2000, 700, torch.from_numpy(keys).to(gpu), 1, L=64)
    runs = []
    for graph in (False, True):
        m = GibbsLDA(c, GibbsConfig(K=100, seed=5, count_mode="auto", auto_switch=5, sampler="mh", use_graph=graph))
        m.initialize()
        m.sweep(2)
        m.sweep(10)
        runs.append(m)
    a, b = runs
    assert b._graph is not None or b._graphs
    assert torch.equal(a.tok_z, b.tok_z) and torch.equal(a.nwk, b.nwk) and torch.equal(a.ndk_cur, b.ndk_cur)


@pytest.mark.parametrize("K,sampler", [(20, "dense"), (50, "dense"), (100, "mh")])
def test_word_init_bitwise_and_seed_free(gpu, K, sampler):
    """ONI_INIT=word: every token of a word starts in the word's hashed topic, on the GPU as in the
    oracle, whatever the seed."""
    tdoc, tword, keys = _toy(300, 400, 9)
    G, KP = ops.choose_tiling(K, "mh" if sampler == "mh" else None)
    cc = build_corpus(tdoc, tword, 300, 400, torch.from_numpy(keys), G, L=64)
    cg = build_corpus(tdoc.to(gpu), tword.to(gpu), 300, 400, torch.from_numpy(keys).to(gpu), G, L=64)
    zs = []
    for seed, c in ((1, cc), (1, cg), (77, cg)):
        m = GibbsLDA(c, GibbsConfig(K=K, seed=seed, use_graph=False, sampler=sampler, init="word"))
        m.initialize()
        zs.append((m.tok_z.cpu(), m.ndk_cur.cpu(), m.nwk.cpu()))
    for i in range(3):
        assert torch.equal(zs[0][i], zs[1][i]) and torch.equal(zs[1][i], zs[2][i])
    w = cc.tok_word.numpy().view(np.uint32)
    real = w != 0xFFFFFFFF
    want = ((spec.mix32(w[real]).astype(np.uint64) * np.uint64(K)) >> np.uint64(32)).astype(np.uint8)
    assert np.array_equal(zs[0][0].numpy()[real], want)


def test_mh_resume_bitwise(gpu):
    """An MH chain restored from its canonical z continues bit for bit (the tables are rebuilt
    from the restored counts every sweep)."""
    tdoc, tword, keys = _toy(400, 300, 13)
    c = build_corpus(tdoc.to(gpu), tword.to(gpu), 400, 300, torch.from_numpy(keys).to(gpu), 1, L=127)
    cfg = dict(K=100, seed=3, sampler="mh")
    a = GibbsLDA(c, GibbsConfig(**cfg))
    a.initialize()
    a.sweep(7)
    b = GibbsLDA(c, GibbsConfig(**cfg))
    b.initialize()
    b.sweep(3)
    z = b.canonical_z().cpu()
    r = GibbsLDA(c, GibbsConfig(**cfg))
    r.load_canonical_z(z, 3)
    r.sweep(4)
    assert torch.equal(a.canonical_z(), r.canonical_z())
    assert torch.equal(a.nwk, r.nwk) and torch.equal(a.ndk_cur, r.ndk_cur)
