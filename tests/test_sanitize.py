"""Race/memory-safety checks for host code: the C++ decoders are built with
ASan+UBSan (`tools/build.py --only native --sanitize`) and fed valid inputs plus random
mutations/truncations of them; any sanitizer report fails the test. (GPU sanitizers are not
available on the GPU pool; kernel races are covered by the run-twice / oracle bitwise tests.)"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FUZZ = os.path.join(ROOT, "oni355", "_lib", "bin", "oni-fuzz_asan")


@pytest.fixture(scope="module")
def fuzz_bin():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build.py"), "--only", "native", "--sanitize"],
                       capture_output=True, text=True)
    if r.returncode != 0 or not os.path.exists(FUZZ):
        pytest.skip(f"sanitizer build unavailable: {r.stderr[-400:]}")
    return FUZZ


def _seeds(tmp_path):
    from oni355.io.decoders import write_flow_csv
    from oni355.io.nfcapd import write_nfcapd
    from oni355.synth.dns import generate_dns, write_pcap
    from oni355.synth.flow import generate_flows
    from oni355.synth.proxy import generate_proxy, write_log
    day = generate_flows(300, seed=1)
    write_flow_csv(str(tmp_path / "f.csv"), day.cols)
    write_nfcapd(str(tmp_path / "nf.lzo"), day.cols, "lzo", per_block=64)
    write_nfcapd(str(tmp_path / "nf.lz4"), day.cols, "lz4", per_block=64)
    write_pcap(generate_dns(200, seed=1), str(tmp_path / "d.pcap"))
    write_log(generate_proxy(200, seed=1), str(tmp_path / "p.log"))
    return {"csv": tmp_path / "f.csv", "nfcapd": tmp_path / "nf.lzo", "pcap": tmp_path / "d.pcap",
            "proxy": tmp_path / "p.log"}


def _run(fuzz_bin, mode, path):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=99",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")
    r = subprocess.run([fuzz_bin, mode, str(path)], capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode == 0, f"{mode} {path}: rc={r.returncode}\n{r.stderr[-2000:]}"


def test_decoders_under_asan(fuzz_bin, tmp_path):
    seeds = _seeds(tmp_path)
    rng = np.random.default_rng(0)
    for mode, p in seeds.items():
        _run(fuzz_bin, mode, p)
        raw = p.read_bytes()
        for k in range(12):
            b = bytearray(raw)
            if k % 3 == 0:
                b = b[: rng.integers(0, len(b))]
            else:
                for _ in range(int(rng.integers(1, 40))):
                    b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            q = tmp_path / f"m_{mode}_{k}"
            q.write_bytes(bytes(b))
            _run(fuzz_bin, mode, q)
    for mode in ("lzo", "lz4"):
        for k in range(20):
            q = tmp_path / f"r_{mode}_{k}"
            q.write_bytes(rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes())
            _run(fuzz_bin, mode, q)
