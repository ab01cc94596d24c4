"""Pinned staging ring (csrc/kernels/stage.hip, oni355/io/staging.py): host → HBM uploads."""
import numpy as np
import pytest
import torch

from oni355.io import staging


def test_cpu_target_returns_host_values():
    a = np.arange(1000, dtype=np.uint32)
    t = staging.upload(a, "cpu", torch.int64)
    assert t.dtype == torch.int64 and torch.equal(t, torch.arange(1000, dtype=torch.int64))


@pytest.mark.gpu
@pytest.mark.parametrize("m", ["1", "reg"])
def test_staged_upload_bitwise_many_sizes(gpu, monkeypatch, m):
    monkeypatch.setenv("ONI_STAGED_H2D", m)
    rng = np.random.default_rng(3)
    # sizes around the chunk boundary, empty, odd byte counts; > N_BUF chunks so the ring wraps
    cb = staging.CHUNK_BYTES
    for nbytes in (0, 1, 7, 4096, cb - 1, cb, cb + 3, 5 * cb + 11):
        a = rng.integers(0, 256, nbytes, dtype=np.uint8)
        t = staging.upload(a, gpu)
        assert t.device.type == "cuda" and t.dtype == torch.uint8 and t.numel() == nbytes
        assert np.array_equal(t.cpu().numpy(), a)
    before = staging.stats()
    x = rng.standard_normal(3_000_001).astype(np.float32)
    tx = staging.upload(x, gpu)
    # kernels on the same stream are ordered after the queued copies
    s = float(tx.double().sum().item())
    assert s == pytest.approx(float(x.astype(np.float64).sum()), rel=1e-12)
    if m == "1":
        assert staging.stats()["bytes"] - before["bytes"] == x.nbytes
    staging.sync()


@pytest.mark.gpu
@pytest.mark.parametrize("m", ["1", "reg"])
def test_flow_to_device_staged_matches_plain(gpu, monkeypatch, m):
    from oni355.pipeline import flow
    from oni355.synth.flow import generate_flows
    day = generate_flows(200_000, seed=5)
    monkeypatch.setenv("ONI_STAGED_H2D", m)
    got = flow.to_device(day.cols, gpu)
    monkeypatch.setenv("ONI_STAGED_H2D", "0")
    want = flow.to_device(day.cols, gpu)
    for k in want:
        assert got[k].dtype == want[k].dtype and torch.equal(got[k], want[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("nbytes", [1, 15, 16, 4095, 4096 * 257 + 3, 64 << 20])
def test_pull_upload_bitwise(gpu, nbytes):
    """oni_h2d_pull (CUs read the pinned buffer, no DMA engine) == the source bytes; an unaligned
    pinned view falls back to the DMA copy and is still exact."""
    g = torch.Generator().manual_seed(nbytes)
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g).pin_memory()
    out = staging.pull_upload(src, "cuda")
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), src)
    if nbytes > 8192:
        view = src[1:]  # 1-byte offset: not 16-B aligned
        out2 = staging.pull_upload(view, "cuda")
        torch.cuda.synchronize()
        assert torch.equal(out2.cpu(), view)


@pytest.mark.gpu
def test_prefetcher_pull_matches_source(gpu):
    cols = {"a": np.arange(1_000_003, dtype=np.int64), "b": np.arange(77, dtype=np.uint32)}
    specs = {"a": torch.int64, "b": torch.int32}
    pinned = staging.Prefetcher.pin(cols, specs)
    pf = staging.Prefetcher("cuda")
    pf.submit(pinned)
    got = pf.take()
    torch.cuda.synchronize()
    assert torch.equal(got["a"].cpu(), torch.from_numpy(cols["a"]))
    assert torch.equal(got["b"].cpu(), torch.from_numpy(cols["b"].view(np.int32)))
    assert pf.copy_ms() >= 0


@pytest.mark.gpu
def test_push_to_host_kernel_readback(gpu):
    src = torch.arange(-5, 1000, dtype=torch.int32, device="cuda") * 7
    dst = torch.zeros(src.numel(), dtype=torch.int32, pin_memory=True)
    staging.push_to_host(src, dst)
    ev = torch.cuda.Event()
    ev.record()
    ev.synchronize()
    assert torch.equal(dst, src.cpu())
    f = torch.randn(33, device="cuda")
    fd = torch.empty(33, pin_memory=True)
    staging.push_to_host(f, fd)
    torch.cuda.synchronize()
    assert torch.equal(fd, f.cpu())


def test_host_ahead_produces_in_order_one_ahead():
    calls = []

    def produce(tag):
        calls.append(tag)
        return len(calls)

    ah = staging.HostAhead(produce, "day")
    assert ah.take() == 1
    assert ah.take() == 2  # the second item was started when the first was taken
    ah.close()
    assert calls[:2] == ["day", "day"]
