"""The dense burn-in → MH hand-over (pipeline.common.build_and_train): the MH model loads the dense
chain's canonical z, and copying the dense model's count tables (GibbsLDA.load_canonical_z's
``counts_from``) gives the tables a recount from z gives, so the MH chain that follows is the same.
CPU here; the GPU case (every count mode the dense model runs) is test_handover_copy_equals_recount_gpu."""
import numpy as np
import pytest
import torch

from oni355.models.corpus import build_corpus
from oni355.models.gibbs import GibbsConfig, GibbsLDA, tiling_for


def _toy(n_docs, V, seed):
    r = np.random.default_rng(seed)
    lens = r.zipf(1.6, n_docs).clip(1, 2000)
    lens[0] = 3000  # one document over many chunks
    tdoc = np.repeat(np.arange(n_docs), lens)
    tword = (r.zipf(1.3, tdoc.size) - 1) % V
    keys = ((np.arange(n_docs, dtype=np.int64) * 2654435761 + seed) % (2**31 - 1)).astype(np.int32)
    return torch.from_numpy(tdoc).to(torch.int32), torch.from_numpy(tword).to(torch.int32), torch.from_numpy(keys)


def _handover(dev, K, burn, after):
    tdoc, tword, keys = _toy(300, 250, K)
    mk = lambda s: build_corpus(tdoc.to(dev), tword.to(dev), 300, 250, keys.to(dev), tiling_for(K, s)[0], L=64)
    dense = GibbsLDA(mk("dense"), GibbsConfig(K=K, seed=77, sampler="dense"))
    dense.initialize()
    dense.sweep(burn)
    z = dense.canonical_z()
    out = []
    for src in (dense, None):
        m = GibbsLDA(mk("mh"), GibbsConfig(K=K, seed=77, sampler="mh"))
        m.load_canonical_z(z, burn, counts_from=src)
        tabs = [m.nwk.clone(), m.ndk[0].clone(), m.nk[0].clone(), m.tok_z.clone()]
        m.sweep(after)
        out.append((tabs, m.canonical_z().cpu(), m.log_likelihood()))
    (ta, za, la), (tb, zb, lb) = out
    for x, y in zip(ta, tb):
        assert torch.equal(x, y)
    assert torch.equal(za, zb) and la == lb
    assert tiling_for(K, "dense") != tiling_for(K, "mh")


@pytest.mark.parametrize("K", [40, 100])
def test_handover_copy_equals_recount(K):
    _handover(torch.device("cpu"), K, 3, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [40, 100])
def test_handover_copy_equals_recount_gpu(gpu, K):
    # 12 dense sweeps: the auto count mode has left "recount" for a delta mode by then
    _handover(gpu, K, 12, 3)


def test_explicit_chunk_len_128_clamped_for_mh():
    """CHUNK_LEN = 128 is valid for the dense kernels; a K = 100 (MH) day clamps it to the MH limit
    instead of failing."""
    from oni355.pipeline.common import build_and_train
    from oni355.ref import spec
    tdoc, tword, keys = _toy(120, 90, 3)
    doc_keys = keys.to(torch.int64)[tdoc.long()]
    vocab = torch.arange(90, dtype=torch.int64)
    msgs = []
    run = build_and_train(doc_keys, vocab[tword.long()], None, vocab, 100, None, 0.01, 5, 6, 128, None,
                          log=msgs.append)
    assert run.corpus.L <= spec.MH_MAX_CHUNK and run.model.mh
    assert any("MH sampler" in m for m in msgs)
    assert run.model.chain["sampler"] == "mh" and run.model.chain["mh_burn"] == 6
