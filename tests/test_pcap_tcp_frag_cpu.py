"""pcap DNS decoder (csrc/io/pcap_dns.cpp): DNS over TCP (length-prefixed messages inside one
segment) and IPv4-fragmented UDP responses reassembled across the parallel decode's chunks, rows
in packet order; split TCP messages and incomplete datagrams are counted, not decoded."""
import struct

import numpy as np
import pytest

from oni355.io.decoders import read_pcap_dns


def _dns_response(qid: int, name: str, qtype: int = 1, answers=(), pad: int = 0) -> bytes:
    q = b"".join(bytes([len(l)]) + l.encode() for l in name.split(".")) + b"\0"
    msg = struct.pack(">HHHHHH", qid, 0x8180, 1, len(answers), 0, 0) + q + struct.pack(">HH", qtype, 1)
    for ip in answers:
        msg += b"\xc0\x0c" + struct.pack(">HHIH", 1, 1, 60, 4) + bytes(int(x) for x in ip.split("."))
    return msg + b"\0" * pad


def _ipv4(src, dst, proto, payload, ident=1, frag_off=0, more=False):
    ff = (0x2000 if more else 0) | (frag_off // 8)
    hdr = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + len(payload), ident, ff, 64, proto, 0,
                      bytes(int(x) for x in src.split(".")), bytes(int(x) for x in dst.split(".")))
    return hdr + payload


def _eth(ip: bytes) -> bytes:
    return b"\x00" * 12 + b"\x08\x00" + ip


def _udp(sport, dport, data):
    return struct.pack(">HHHH", sport, dport, 8 + len(data), 0) + data


def _tcp(sport, dport, data):
    return struct.pack(">HHIIBBHHH", sport, dport, 1, 1, 5 << 4, 0x18, 65535, 0, 0) + data


def _write(path, frames):
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xa1b2c3d4, 2, 4, 0, 0, 65535, 1))
        for i, fr in enumerate(frames):
            f.write(struct.pack("<IIII", 1467936000 + i, 0, len(fr), len(fr)))
            f.write(fr)


def test_tcp_messages_and_fragment_reassembly(tmp_path):
    srv, cli = "10.0.0.53", "10.1.2.3"
    big = _udp(53, 5555, _dns_response(7, "big.example.com", answers=["1.2.3.4"], pad=900))
    f1, f2, f3 = big[:400], big[400:800], big[800:]
    frames = [
        _eth(_ipv4(srv, cli, 17, _udp(53, 4000, _dns_response(1, "a.example.com", answers=["9.9.9.9"])))),   # 0
        _eth(_ipv4(srv, cli, 6, _tcp(53, 4001, b"".join(struct.pack(">H", len(m)) + m for m in (
            _dns_response(2, "t1.example.org", qtype=16), _dns_response(3, "t2.example.org")))))),      # 1: 2 msgs
        _eth(_ipv4(srv, cli, 17, f3, ident=77, frag_off=800)),                                          # 2 (last)
        _eth(_ipv4(srv, cli, 17, f1, ident=77, frag_off=0, more=True)),                                 # 3
        _eth(_ipv4(srv, cli, 6, _tcp(53, 4002, struct.pack(">H", 300) + b"\x00" * 40))),                # 4 partial
        _eth(_ipv4(srv, cli, 17, f2, ident=77, frag_off=400, more=True)),                               # 5 completes
        _eth(_ipv4(srv, cli, 17, big[:400], ident=99, frag_off=0, more=True)),                          # 6 no tail
        _eth(_ipv4(srv, cli, 17, _udp(53, 4003, _dns_response(4, "z.example.net"))))                     # 7
    ]
    p = str(tmp_path / "x.pcap")
    _write(p, frames)
    for threads in (1, 3):
        c = read_pcap_dns(p, threads=threads)
        names = c["dns_qry_name"].to_list()
        assert names == ["a.example.com", "t1.example.org", "t2.example.org", "big.example.com", "z.example.net"]
        assert c["dns_qry_type"].tolist() == [1, 16, 1, 1, 1]
        assert c["dns_a"].to_list()[3] == "1.2.3.4"
        # the reassembled datagram carries the frame that completed it (packet 5)
        assert c["unix_tstamp"].tolist() == [1467936000, 1467936001, 1467936001, 1467936005, 1467936007]
        assert c["_tcp_partial"] == 1 and c["_frag_incomplete"] == 1


def test_frame_time_is_formatted_only_for_rendered_rows(tmp_path):
    """pcap frame_time text is lazy: rendering the result rows formats just those rows (formatting
    every packet's time cost 0.27 s per 2M-packet day)."""
    from oni355.io import results as rio
    from oni355.io.decoders import FrameTimeColumn, frame_times
    from oni355.synth.dns import generate_dns, write_pcap
    day = generate_dns(3000, seed=5)
    p = str(tmp_path / "d.pcap")
    write_pcap(day, p)
    cols = read_pcap_dns(p)
    ft = cols["frame_time"]
    assert isinstance(ft, FrameTimeColumn)
    rows = np.array([5, 17, 2999])
    r = rio.format_events("dns", cols, rows, ["w"] * 3, np.zeros(3, np.float32))
    assert ft._mat is None
    want = frame_times(ft.ts_ns[rows]).to_list()
    import csv
    assert [row[0] for row in csv.reader(ln.decode() for ln in r.lines())] == want


def _write_ts(path, frames_ts):
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xa1b2c3d4, 2, 4, 0, 0, 65535, 1))
        for ts, fr in frames_ts:
            f.write(struct.pack("<IIII", ts, 0, len(fr), len(fr)))
            f.write(fr)


def test_fragments_reusing_an_ip_id_are_separate_datagrams(tmp_path):
    """The 16-bit IP id wraps in a day-long capture: two fragmented responses between the same
    hosts with the same id are two datagrams (the repeated offset opens the second), and pieces
    more than 30 s of frame time apart never join one datagram."""
    srv, cli = "10.0.0.53", "10.1.2.3"
    a = _udp(53, 5000, _dns_response(11, "first.example.com", answers=["1.1.1.1"], pad=600))
    b = _udp(53, 5001, _dns_response(12, "second.example.com", answers=["2.2.2.2"], pad=600))
    t0 = 1467936000
    frames = [
        (t0, _eth(_ipv4(srv, cli, 17, a[:400], ident=5, frag_off=0, more=True))),
        (t0 + 1, _eth(_ipv4(srv, cli, 17, a[400:], ident=5, frag_off=400))),
        (t0 + 2, _eth(_ipv4(srv, cli, 17, b[:400], ident=5, frag_off=0, more=True))),
        (t0 + 3, _eth(_ipv4(srv, cli, 17, b[400:], ident=5, frag_off=400))),
        # id 6: head, then its tail 40 s later -> two incomplete groups, no row
        (t0 + 4, _eth(_ipv4(srv, cli, 17, a[:400], ident=6, frag_off=0, more=True))),
        (t0 + 44, _eth(_ipv4(srv, cli, 17, a[400:], ident=6, frag_off=400))),
        # id 7: a head whose datagram never completes, then a full datagram with the same id
        (t0 + 45, _eth(_ipv4(srv, cli, 17, b[:400], ident=7, frag_off=0, more=True))),
        (t0 + 46, _eth(_ipv4(srv, cli, 17, a[:400], ident=7, frag_off=0, more=True))),
        (t0 + 47, _eth(_ipv4(srv, cli, 17, a[400:], ident=7, frag_off=400))),
    ]
    p = str(tmp_path / "wrap.pcap")
    _write_ts(p, frames)
    for threads in (1, 4):
        c = read_pcap_dns(p, threads=threads)
        assert c["dns_qry_name"].to_list() == ["first.example.com", "second.example.com", "first.example.com"]
        assert c["dns_a"].to_list() == ["1.1.1.1", "2.2.2.2", "1.1.1.1"]
        assert c["unix_tstamp"].tolist() == [t0 + 1, t0 + 3, t0 + 47]
        assert c["_frag_incomplete"] == 3


def test_duplicate_fragment_is_dropped_not_a_new_datagram(tmp_path):
    """Mirror / SPAN captures repeat packets: an exact copy of a fragment the open datagram already
    holds (f0, f1, f1', f2) is dropped, as tshark's reassembly does; the datagram still completes."""
    srv, cli = "10.0.0.53", "10.1.2.3"
    big = _udp(53, 5555, _dns_response(9, "dup.example.com", answers=["5.6.7.8"], pad=900))
    f0, f1, f2 = big[:400], big[400:800], big[800:]
    t0 = 1467936000
    frames = [
        (t0, _eth(_ipv4(srv, cli, 17, f0, ident=31, frag_off=0, more=True))),
        (t0, _eth(_ipv4(srv, cli, 17, f1, ident=31, frag_off=400, more=True))),
        (t0 + 1, _eth(_ipv4(srv, cli, 17, f1, ident=31, frag_off=400, more=True))),  # duplicate
        (t0 + 2, _eth(_ipv4(srv, cli, 17, f2, ident=31, frag_off=800))),
    ]
    p = str(tmp_path / "dup.pcap")
    _write_ts(p, frames)
    for threads in (1, 2):
        c = read_pcap_dns(p, threads=threads)
        assert c["dns_qry_name"].to_list() == ["dup.example.com"]
        assert c["dns_a"].to_list() == ["5.6.7.8"]
        assert c["unix_tstamp"].tolist() == [t0 + 2]
        assert c["_frag_incomplete"] == 0


def test_parallel_index_equals_sequential_walk(tmp_path):
    """The classic-pcap index runs in parallel byte ranges with speculated record starts, stitched
    exactly: any thread count gives the sequential walk's packets -- including payloads that
    imitate record headers (a UDP payload carrying copies of pcap record headers) and a truncated
    final record."""
    import numpy as np
    from oni355.synth.dns import generate_dns, write_pcap
    day = generate_dns(3000, seed=9)
    p = str(tmp_path / "d.pcap")
    write_pcap(day, p)
    ref = read_pcap_dns(p, threads=1)
    for th in (2, 3, 7, 16, 64):
        got = read_pcap_dns(p, threads=th)
        for k in ("unix_tstamp", "frame_len", "ip_src", "ip_dst", "dns_qry_type", "dns_qry_rcode"):
            assert np.array_equal(ref[k], got[k]), (th, k)
        assert ref["dns_qry_name"].to_list() == got["dns_qry_name"].to_list()
        assert got["_packets"] == ref["_packets"]
    # decoys: payloads full of plausible record headers, then a truncated tail record
    srv, cli = "10.0.0.53", "10.1.2.3"
    decoy = struct.pack("<IIII", 1467936000, 0, 40, 40) * 24
    frames = []
    for i in range(400):
        if i % 3 == 0:
            frames.append((1467936000 + i, _eth(_ipv4(srv, cli, 17, _udp(9999, 9999, decoy)))))
        else:
            frames.append((1467936000 + i, _eth(_ipv4(srv, cli, 17, _udp(53, 4000 + i, _dns_response(
                i, f"h{i}.example.com", answers=["9.9.9.9"]))))))
    q = str(tmp_path / "decoy.pcap")
    _write_ts(q, frames)
    with open(q, "ab") as f:
        f.write(struct.pack("<IIII", 1467937000, 0, 500, 500) + b"\x00" * 100)  # truncated record
    ref = read_pcap_dns(q, threads=1)
    assert ref["_packets"] == 400
    for th in (2, 5, 13, 32):
        got = read_pcap_dns(q, threads=th)
        assert got["_packets"] == 400
        assert got["dns_qry_name"].to_list() == ref["dns_qry_name"].to_list()
        assert np.array_equal(got["unix_tstamp"], ref["unix_tstamp"])
