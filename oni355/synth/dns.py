"""Seeded synthetic DNS-response day (+ a synthetic top-1M list) with planted tunnelling/DGA.

Documents are client IPs (``ip_dst`` of responses, as in ONI's DNS model); each client has a
behaviour-profile mix θ* ~ Dir(alpha_true). Profiles differ in domains, subdomain style (none /
``www``-like / CDN hex / service labels / reverse-PTR), query type, rcode mix and time of day.
Planted anomalies: long high-entropy subdomains of a rare domain, TXT/NULL queries at night
(DNS tunnelling / DGA shape). ``write_pcap`` serialises the day through our own pcap writer so
the C++ pcap decoder (the tshark replacement) is exercised end to end.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..store.columnar import StringColumn

_POPULAR = ["google.com", "youtube.com", "facebook.com", "amazon.com", "wikipedia.org", "twitter.com", "yahoo.com",
            "bing.com", "linkedin.com", "netflix.com", "microsoft.com", "apple.com", "github.com", "office.com",
            "bbc.co.uk", "spiegel.de", "amazon.co.jp", "baidu.com", "reddit.com", "instagram.com"]
_CDN = ["cloudfront.net", "akamaiedge.net", "fastly.net", "azureedge.net", "edgecastcdn.net"]
_MAIL = ["outlook.com", "gmail.com", "mimecast.com", "pphosted.com"]
_TELEM = ["telemetry.microsoft.com", "metrics.icloud.com", "app-measurement.com", "crashlytics.com"]
_SERVICE = ["_ldap._tcp.dc._msdcs", "_kerberos._udp", "_sip._tls", "_xmpp-client._tcp"]
_WORDS = ["www", "mail", "api", "cdn", "static", "img", "login", "m", "news", "docs", "drive", "accounts", "ads",
          "video", "update", "portal", "app", "auth", "store", "support"]

# (name, domain-pool key, subdomain style, qtypes, qtype weights, nx-rate, peak hour, hour sd)
_PROFILES = [
    ("browse", "popular", "word", [1, 28], [0.7, 0.3], 0.01, 14, 4.0),
    ("cdn", "cdn", "hex", [1, 28], [0.8, 0.2], 0.0, 20, 3.0),
    ("mail", "mail", "word", [15, 1], [0.5, 0.5], 0.02, 9, 2.0),
    ("internal", "user", "word", [1, 33], [0.8, 0.2], 0.05, 11, 3.0),
    ("reverse", "ptr", "ptr", [12], [1.0], 0.2, 12, 6.0),
    ("service", "user", "service", [33], [1.0], 0.1, 8, 2.0),
    ("telemetry", "telem", "hex", [1], [1.0], 0.0, 3, 6.0),
    ("browse-night", "popular", "word", [1, 28, 5], [0.6, 0.3, 0.1], 0.02, 22, 2.0),
]


@dataclass
class DnsDay:
    cols: dict
    top_domains: list[str]
    anomaly_rows: np.ndarray
    theta_true: np.ndarray
    # generating label per row (tools/oracle_recall.py): profile p, len(profiles) + b for long-tail
    # behaviour b, -1 for a planted anomaly
    labels: np.ndarray | None = None

    @property
    def n(self) -> int:
        return int(len(self.cols["ip_dst"]))


def _hex(rng, n, lo, hi):
    ln = rng.integers(lo, hi + 1, size=n)
    alphabet = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
    return ["".join(map(chr, alphabet[rng.integers(0, 16, size=k)])) for k in ln]


def top_domain_list(n_extra: int = 2000, seed: int = 1) -> list[str]:
    rng = np.random.default_rng(seed)
    tl = ["com", "net", "org", "de", "co.uk", "io", "info", "jp"]
    extra = [f"site{i}{'abcdefgh'[i % 8]}.{tl[rng.integers(0, len(tl))]}" for i in range(n_extra)]
    return _POPULAR + _CDN + _MAIL + ["microsoft.com", "icloud.com", "app-measurement.com", "crashlytics.com"] + extra


# long-tail record types / rcodes of a real resolver day (A, AAAA, PTR, MX, SRV, CNAME, NS, SOA, HTTPS,
# SVCB, DS, DNSKEY, NAPTR, CAA, TLSA) with Zipf-like weights
# (the planted queries' record types, _ANOMALY_QTYPES, are kept out of the long tail: a planted query
# stays an individually rare word on the realistic day)
_ANOMALY_QTYPES = [16, 10, 13, 17, 29, 99, 252, 255]
_WIDE_QTYPES = [1, 28, 12, 15, 33, 5, 2, 6, 65, 64, 43, 48, 35, 257, 52]
_WIDE_RCODES = [0, 3, 2, 5, 1, 4]
_ALPHABETS = [b"abcdefghijklmnopqrstuvwxyz", b"0123456789abcdef", b"abcdefghijklmnopqrstuvwxyz0123456789-",
              b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789"]


def _wide_names(rng, m: int, domains: list[str]) -> list[str]:
    """Names of every shape: 0-5 labels of 1-24 characters over alphabets of 16-62 symbols under a
    Zipf-chosen registered domain (subdomain length / entropy / period quintiles all spread)."""
    nlab = rng.integers(0, 6, size=m)
    dz = 1.0 / np.arange(1, len(domains) + 1)
    dsel = rng.choice(len(domains), size=m, p=dz / dz.sum())
    alph = rng.integers(0, len(_ALPHABETS), size=m)
    out = []
    for j in range(m):
        a = np.frombuffer(_ALPHABETS[alph[j]], dtype=np.uint8)
        labs = [bytes(a[rng.integers(0, a.size, size=int(rng.integers(1, 25)))]).decode() for _ in range(nlab[j])]
        out.append(".".join(labs + [domains[dsel[j]]]))
    return out


def generate_dns(n: int, seed: int = 5, n_clients: int | None = None, user_domain: str = "intel",
                 alpha_true: float = 0.1, n_anomalies: int | None = None, rank: int = 0,
                 date_unix: int = 1467936000, wide_vocab: float = 0.0, anomaly_kind: str = "rare") -> DnsDay:
    """``wide_vocab``: fraction of (non-anomalous) rows drawn from the long tail instead of a
    behaviour profile -- any of 18 record types and 6 rcodes, names of every shape under ~2000
    domains, any hour -- which takes the day's vocabulary from ~4k words to ~1e5 (the sizing of
    SURVEY.md §7.5)."""
    rng = np.random.default_rng([seed, rank])
    hrng = np.random.default_rng([seed, 0xD5])
    P = len(_PROFILES)
    if n_clients is None:
        n_clients = max(32, n // 40)
    if n_anomalies is None:
        n_anomalies = max(5, min(200, n // 20000))
    theta = hrng.dirichlet(np.full(P, alpha_true), size=n_clients)
    w = 1.0 / np.power(np.arange(1, n_clients + 1), 1.1)
    w = w[hrng.permutation(n_clients)]
    w /= w.sum()
    cli = rng.choice(n_clients, size=n, p=w)
    cum = np.cumsum(theta, axis=1)
    cum[:, -1] = 1
    z = np.clip(np.searchsorted((cum + np.arange(n_clients)[:, None]).ravel(), cli + rng.random(n), side="right")
                - cli * P, 0, P - 1)
    labels = z.astype(np.int32)
    pools = {"popular": _POPULAR, "cdn": _CDN, "mail": _MAIL, "telem": _TELEM,
             "user": [f"corp.{user_domain}.com", f"{user_domain}.com", f"eng.{user_domain}.com"]}
    names = [""] * n
    qtype = np.zeros(n, np.int32)
    rcode = np.zeros(n, np.int32)
    hour_f = np.zeros(n)
    for k, (_, pool, style, qts, qw, nx, peak, hsd) in enumerate(_PROFILES):
        idx = np.nonzero(z == k)[0]
        m = idx.size
        if not m:
            continue
        qtype[idx] = rng.choice(qts, size=m, p=np.asarray(qw) / np.sum(qw))
        rcode[idx] = np.where(rng.random(m) < nx, 3, 0)
        hour_f[idx] = rng.normal(peak, hsd, size=m)
        if style == "ptr":
            octs = rng.integers(0, 256, size=(m, 4))
            for j, i in enumerate(idx):
                names[i] = f"{octs[j, 0]}.{octs[j, 1]}.{octs[j, 2]}.10.in-addr.arpa"
            continue
        doms = pools[pool]
        dz = 1.0 / np.arange(1, len(doms) + 1)
        dsel = rng.choice(len(doms), size=m, p=dz / dz.sum())
        if style == "word":
            subs = [_WORDS[j] for j in rng.integers(0, len(_WORDS), size=m)]
            for j, i in enumerate(idx):
                names[i] = f"{subs[j]}.{doms[dsel[j]]}"
        elif style == "hex":
            hx = _hex(rng, m, 6, 14)
            for j, i in enumerate(idx):
                names[i] = f"{hx[j]}.{doms[dsel[j]]}"
        elif style == "service":
            sv = rng.integers(0, len(_SERVICE), size=m)
            for j, i in enumerate(idx):
                names[i] = f"{_SERVICE[sv[j]]}.{doms[dsel[j]]}"
    if wide_vocab > 0:
        # long-tail rows come from a codebook of ~n/100 query behaviours (name shape, record type,
        # rcode, hour); every client owns ⌈its long-tail rows / 8⌉ of them (dealt round-robin, so
        # each has several owners) and repeats them, as synth.flow's realistic day does.
        # Independent per-row draws made every other long-tail row a day-unique word, and uniform
        # draws from the codebook scattered each behaviour over unrelated clients -- either way
        # P(word | doc) could not tell them from a planted query
        wide = np.nonzero(rng.random(n) < wide_vocab)[0]
        m = wide.size
        crng = np.random.default_rng([seed, 0xC0DE])
        W = max(200, n // 100)
        qz = 1.0 / np.arange(1, len(_WIDE_QTYPES) + 1) ** 1.2
        cb_q = crng.choice(_WIDE_QTYPES, size=W, p=qz / qz.sum())
        rz = np.array([0.8, 0.1, 0.05, 0.03, 0.015, 0.005])
        cb_r = crng.choice(_WIDE_RCODES, size=W, p=rz / rz.sum())
        cb_h = crng.uniform(0, 24, size=W)
        cb_n = _wide_names(crng, W, top_domain_list())
        c_w = cli[wide]
        slots = np.clip(-(-np.bincount(c_w, minlength=n_clients) // 8), 1, 64)
        first = np.concatenate([[0], np.cumsum(slots)[:-1]])
        orng = np.random.default_rng([seed, 0x0515])
        n_sl = int(slots.sum())
        own = np.concatenate([orng.permutation(W) for _ in range(-(-n_sl // W))])[:n_sl]
        own = own[orng.permutation(n_sl)]
        b = own[first[c_w] + (rng.random(m) * slots[c_w]).astype(np.int64)]
        labels[wide] = P + b
        qtype[wide] = cb_q[b]
        rcode[wide] = cb_r[b]
        hour_f[wide] = cb_h[b]
        for i, j in zip(wide.tolist(), b.tolist()):
            names[i] = cb_n[j]
    hour = np.mod(np.floor(hour_f), 24).astype(np.int64)
    # planted tunnelling / DGA
    anomaly_rows = np.sort(rng.choice(n, size=min(n_anomalies, n), replace=False))
    labels[anomaly_rows] = -1
    if anomaly_rows.size:
        quiet = np.argsort(w)[: max(1, n_clients // 10)]
        q_draw = quiet[rng.integers(0, quiet.size, size=anomaly_rows.size)]
        # "rare": planted on the least active tenth of the clients; "rare-active": on the row's own
        # (activity-drawn) client
        if anomaly_kind == "rare":
            cli[anomaly_rows] = q_draw
        # each anomaly is an individually rare behaviour (tunnel/DGA-like name of varying shape, odd
        # record type, odd hour): a hundred copies of ONE pattern would form a topic of their own
        # and stop being rare for the model at large day sizes
        na = anomaly_rows.size
        hx = _hex(rng, na, 20, 72)
        nlab = rng.integers(1, 4, size=na)
        for j, i in enumerate(anomaly_rows):
            h, k = hx[j], int(nlab[j])
            cut = np.linspace(0, len(h), k + 1).astype(int)
            sub = ".".join(h[cut[t]:cut[t + 1]] for t in range(k))
            names[i] = f"{sub}.x{rng.integers(100, 999)}tunnel.biz"
        qtype[anomaly_rows] = rng.choice(_ANOMALY_QTYPES, size=na)
        rcode[anomaly_rows] = rng.choice([0, 2, 5], size=na)
        hour[anomaly_rows] = rng.integers(1, 6, size=na)
    minute = rng.integers(0, 60, size=n)
    sec = rng.integers(0, 60, size=n)
    unix = date_unix + hour * 3600 + minute * 60 + sec
    n_ans = np.where((rcode == 0) & np.isin(qtype, [1]), rng.integers(1, 4, size=n), 0).astype(np.int32)
    name_len = np.array([len(s) for s in names], dtype=np.int64)
    frame_len = (14 + 20 + 8 + 12 + name_len + 2 + 4 + 16 * n_ans).astype(np.int32)
    client_ip = (np.uint32(10) << np.uint32(24)) | (np.uint32(1) << np.uint32(16)) | cli.astype(np.uint32)
    server_ip = np.full(n, (10 << 24) | (0 << 16) | (0 << 8) | 53, dtype=np.uint32)
    answer = (np.uint32(93) << np.uint32(24)) | rng.integers(0, 1 << 24, size=n).astype(np.uint32)
    def _ip(v):
        v = int(v) & 0xFFFFFFFF
        return f"{v >> 24}.{(v >> 16) & 255}.{(v >> 8) & 255}.{v & 255}"

    a_str = [""] * n
    for i in np.nonzero(n_ans)[0].tolist():
        a_str[i] = ",".join(_ip(int(answer[i]) + k) for k in range(int(n_ans[i])))
    cols = {
        "frame_time": StringColumn.from_list([""] * n),
        "unix_tstamp": unix.astype(np.int64),
        "frame_len": frame_len,
        "ip_src": server_ip,
        "ip_dst": client_ip.astype(np.uint32),
        "dns_qry_name": StringColumn.from_list(names),
        "dns_qry_type": qtype,
        "dns_qry_class": np.ones(n, np.int32),
        "dns_qry_rcode": rcode,
        "dns_a": StringColumn.from_list(a_str),
        "_n_answers": n_ans,
        "_answer_ip": answer,
    }
    return DnsDay(cols=cols, top_domains=top_domain_list(), anomaly_rows=anomaly_rows, theta_true=theta,
                  labels=labels)


def write_pcap(day: DnsDay, path: str) -> int:
    from ..io.decoders import write_pcap_dns
    c = day.cols
    return write_pcap_dns(path, c["unix_tstamp"].astype(np.int64) * 1_000_000_000, c["ip_src"], c["ip_dst"],
                          c["dns_qry_name"], c["dns_qry_type"], c["dns_qry_rcode"], c["_n_answers"], c["_answer_ip"])
