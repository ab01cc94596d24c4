"""Seeded synthetic web-proxy day (Bluecoat access-log fields) with planted anomalies.

Documents are client IPs; profiles differ in hosts, methods, content types, user agents, URI
shapes and time of day. Planted anomalies: rare user agent + POST of long high-entropy URIs to a
non-top host at night (C2 beaconing / exfiltration shape). :func:`write_log` renders the day as a
Bluecoat ``#Fields:`` access log so the C++ log tokenizer is exercised end to end.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..store.columnar import StringColumn

_UAS = ["Mozilla/5.0 (Windows NT 10.0; Win64; x64) AppleWebKit/537.36 Chrome/51.0 Safari/537.36",
        "Mozilla/5.0 (Macintosh; Intel Mac OS X 10_11_5) AppleWebKit/601.6.17 Safari/601.6.17",
        "Mozilla/5.0 (Windows NT 6.1; Trident/7.0; rv:11.0) like Gecko",
        "Microsoft-CryptoAPI/6.1", "Windows-Update-Agent/7.9", "curl/7.47.0", "okhttp/3.2.0",
        "Mozilla/5.0 (iPhone; CPU iPhone OS 9_3 like Mac OS X) Mobile/13E238"]
_HOSTS = {"web": ["www.google.com", "www.bbc.co.uk", "en.wikipedia.org", "www.amazon.com", "news.yahoo.com"],
          "cdn": ["d1.cloudfront.net", "a248.e.akamai.net", "static.xx.fbcdn.net"],
          "update": ["download.windowsupdate.com", "ctldl.windowsupdate.com", "swcdn.apple.com"],
          "api": ["api.github.com", "graph.facebook.com", "api.twitter.com"],
          "video": ["r3---sn.googlevideo.com", "video.twimg.com"]}
_CTYPES = {"web": ["text/html", "text/css", "application/javascript", "image/png"],
           "cdn": ["image/jpeg", "image/gif", "application/javascript"],
           "update": ["application/octet-stream", "application/x-cab-compressed"],
           "api": ["application/json"], "video": ["video/mp4"]}
_PROFILES = [  # (hosts, methods, method weights, ua indices, peak hour, hour sd)
    ("web", ["GET", "POST"], [0.9, 0.1], [0, 1, 2, 7], 13, 3.5),
    ("cdn", ["GET"], [1.0], [0, 1, 2, 7], 14, 4.0),
    ("update", ["GET", "HEAD"], [0.8, 0.2], [3, 4], 3, 2.0),
    ("api", ["GET", "POST", "PUT"], [0.6, 0.3, 0.1], [5, 6], 11, 4.0),
    ("video", ["GET"], [1.0], [0, 1, 7], 20, 2.0),
]

PROXY_FIELDS = ["date", "time", "time-taken", "c-ip", "cs-username", "cs-auth-group", "x-exception-id",
                "sc-filter-result", "cs-categories", "cs(Referer)", "sc-status", "s-action", "cs-method",
                "rs(Content-Type)", "cs-uri-scheme", "cs-host", "cs-uri-port", "cs-uri-path", "cs-uri-query",
                "cs-uri-extension", "cs(User-Agent)", "s-ip", "sc-bytes", "cs-bytes", "x-virus-id"]


@dataclass
class ProxyDay:
    cols: dict
    anomaly_rows: np.ndarray
    # generating label per row (tools/oracle_recall.py): profile p, len(profiles) + b for long-tail
    # behaviour b, -1 for a planted anomaly
    labels: np.ndarray | None = None

    @property
    def n(self) -> int:
        return int(len(self.cols["clientip"]))


N_TEMPLATES = 24  # request templates per behaviour profile

# the planted requests' methods (_ANOMALY_METHODS) are kept out of the long tail, as synth.flow keeps
# its anomaly ports out: a planted request stays an individually rare word on the realistic day
_ANOMALY_METHODS = ["CONNECT", "DELETE", "PROPFIND", "OPTIONS"]
_WIDE_METHODS = ["GET", "POST", "HEAD", "PUT", "PATCH", "TRACE"]
_WIDE_CTYPES = ["text/html", "text/plain", "text/css", "text/javascript", "image/png", "image/jpeg", "image/gif",
                "image/webp", "application/javascript", "application/json", "application/xml", "application/pdf",
                "application/octet-stream", "application/zip", "application/x-protobuf", "video/mp4", "video/webm",
                "audio/mpeg", "multipart/form-data", "font/woff2", "-", ""]
_WIDE_STATUS = [200, 304, 302, 404, 204, 301, 206, 403, 500, 401, 503, 400, 407, 502, 504, 405, 307, 429, 410, 501]


def _wide_rows(rng, m: int):
    """Long-tail request fields: (host, method, user agent, content type, path, status) per row."""
    mz = 1.0 / np.arange(1, len(_WIDE_METHODS) + 1) ** 1.5
    cz = 1.0 / np.arange(1, len(_WIDE_CTYPES) + 1)
    sz = 1.0 / np.arange(1, len(_WIDE_STATUS) + 1) ** 1.3
    meth = rng.choice(len(_WIDE_METHODS), size=m, p=mz / mz.sum())
    ct = rng.choice(len(_WIDE_CTYPES), size=m, p=cz / cz.sum())
    st = np.asarray(_WIDE_STATUS)[rng.choice(len(_WIDE_STATUS), size=m, p=sz / sz.sum())]
    # ~20k distinct user agents, Zipf: the UA-frequency quintile then spreads over all 5 values
    uz = 1.0 / np.arange(1, 20001) ** 0.9
    uas = rng.choice(20000, size=m, p=uz / uz.sum())
    hosts = rng.integers(0, 50000, size=m)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-_=%", np.uint8)
    plen = rng.integers(1, 160, size=m)
    pk = rng.integers(8, alpha.size + 1, size=m)  # alphabet prefix: path entropy spreads too
    rows = []
    for j in range(m):
        path = "/" + bytes(alpha[rng.integers(0, pk[j], size=int(plen[j]))]).decode()
        rows.append((f"h{hosts[j]}.site{hosts[j] % 997}.com", _WIDE_METHODS[meth[j]],
                     f"Agent/{uas[j] % 97}.{uas[j]} (build {uas[j] * 7919 % 10007})", _WIDE_CTYPES[ct[j]], path,
                     int(st[j])))
    return rows


def generate_proxy(n: int, seed: int = 9, n_clients: int | None = None, alpha_true: float = 0.15,
                   n_anomalies: int | None = None, rank: int = 0, date: str = "2016-07-08",
                   wide_vocab: float = 0.0, anomaly_kind: str = "rare") -> ProxyDay:
    """``anomaly_kind``: "rare" -- individually rare requests (unique UA, odd method / content
    type, long high-entropy URI, night hour) from the least active tenth of the clients;
    "rare-active" -- the same requests from the row's own (activity-drawn) client;
    "offprofile" -- a request of the client's least likely behaviour profile (common words, rare
    for that client).
    ``wide_vocab``: fraction of (non-anomalous) rows drawn from the long tail -- 10 methods, 22
    content types, 20 status codes, ~20k user agents, URIs of every length and alphabet, any hour
    -- instead of a behaviour profile (vocabulary ~4e4 → ~1e5+; SURVEY.md §7.5 sizing)."""
    rng = np.random.default_rng([seed, rank])
    hrng = np.random.default_rng([seed, 0xB1])
    P = len(_PROFILES)
    if n_clients is None:
        n_clients = max(32, n // 50)
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
    # planted rows are chosen first (the long-tail rows below never overwrite them)
    arng = np.random.default_rng([seed, rank, 0xA11])
    anomaly_rows = np.sort(arng.choice(n, size=min(n_anomalies, n), replace=False))
    if anomaly_kind == "offprofile" and anomaly_rows.size:
        # behaviour its client never shows: the row comes from the client's least likely profile
        # (globally common words, rare for this client -- the P(word | doc) anomaly)
        z[anomaly_rows] = np.argmin(theta[cli[anomaly_rows]], axis=1)
    labels = z.astype(np.int32)
    host, method, ua, ctype, path = [""] * n, [""] * n, [""] * n, [""] * n, [""] * n
    hour_f = np.zeros(n)
    status = np.full(n, 200, np.int64)
    # each profile serves N_TEMPLATES request templates (host, path, method, content type,
    # status), drawn Zipf-like: what a page load, an update check or an API call repeats all day.
    # A client keeps one user agent per profile. Independent per-row draws of every field made a
    # 6000-row day ~1200 day-unique words, among which no planted request stood out
    # (profiles/r3/recall_sweep_codebook.jsonl: proxy recall 0.03-0.12).
    trng = np.random.default_rng([seed, 0x7E3])
    tz = 1.0 / np.arange(1, N_TEMPLATES + 1)
    tz /= tz.sum()
    for k, (key, meths, mw, uas, peak, hsd) in enumerate(_PROFILES):
        idx = np.nonzero(z == k)[0]
        m = idx.size
        hs, cts = _HOSTS[key], _CTYPES[key]
        t_host = trng.integers(0, len(hs), N_TEMPLATES)
        t_ct = trng.integers(0, len(cts), N_TEMPLATES)
        t_m = trng.choice(len(meths), size=N_TEMPLATES, p=np.asarray(mw) / np.sum(mw))
        t_path = ["/" + "/".join(f"p{trng.integers(0, 50)}" for _ in range(int(trng.integers(1, 4)))) + ".html"
                  for _ in range(N_TEMPLATES)]
        t_st = np.where(trng.random(N_TEMPLATES) < 0.85, 200, trng.choice([304, 302, 404], size=N_TEMPLATES))
        if not m:
            continue
        tsel = rng.choice(N_TEMPLATES, size=m, p=tz)
        hour_f[idx] = rng.normal(peak, hsd, m)
        status[idx] = t_st[tsel]
        for j, i in enumerate(idx.tolist()):
            t = tsel[j]
            host[i], ctype[i], method[i] = hs[t_host[t]], cts[t_ct[t]], meths[t_m[t]]
            ua[i] = _UAS[uas[(cli[i] * 7 + k) % len(uas)]]
            path[i] = t_path[t]
    if wide_vocab > 0:
        # long-tail rows come from a codebook of ~n/100 request behaviours (host, method, agent,
        # content type, URI, status, hour); every client owns ⌈its long-tail rows / 8⌉ of them
        # (dealt round-robin, so each behaviour has several owners) and repeats them, as
        # synth.flow's realistic day does: a wide vocabulary whose words are common in the
        # documents that carry them
        wide = np.nonzero(rng.random(n) < wide_vocab)[0]
        wide = wide[~np.isin(wide, anomaly_rows)]
        crng = np.random.default_rng([seed, 0xC0DE])
        W = max(200, n // 100)
        cb = _wide_rows(crng, W)
        cb_h = crng.uniform(0, 24, size=W)
        c_w = cli[wide]
        slots = np.clip(-(-np.bincount(c_w, minlength=n_clients) // 8), 1, 64)
        first = np.concatenate([[0], np.cumsum(slots)[:-1]])
        orng = np.random.default_rng([seed, 0x0515])
        n_sl = int(slots.sum())
        own = np.concatenate([orng.permutation(W) for _ in range(-(-n_sl // W))])[:n_sl]
        own = own[orng.permutation(n_sl)]
        b = own[first[c_w] + (rng.random(wide.size) * slots[c_w]).astype(np.int64)]
        hour_f[wide] = cb_h[b]
        labels[wide] = P + b
        for i, j in zip(wide.tolist(), b.tolist()):
            host[i], method[i], ua[i], ctype[i], path[i], status[i] = cb[j]
    hour = np.mod(np.floor(hour_f), 24).astype(int)
    quiet = np.argsort(w)[: max(1, n_clients // 10)]
    # individually rare behaviours (see synth.dns): varying method, content type, URI shape, hour
    a_methods = _ANOMALY_METHODS
    a_ctypes = ["application/x-www-form-urlencoded", "application/octet-stream", "application/x-msdownload",
                "application/x-sh", "text/x-python"]
    for i in anomaly_rows:
        if anomaly_kind == "rare":
            cli[i] = quiet[rng.integers(0, quiet.size)]
        if anomaly_kind == "offprofile":
            continue
        host[i] = f"x{rng.integers(1000, 9999)}.badcdn-sync.biz"
        method[i] = a_methods[rng.integers(0, len(a_methods))]
        ua[i] = f"Mozilla/4.0 (compatible; agent-{rng.integers(10**6, 10**7)})"
        ctype[i] = a_ctypes[rng.integers(0, len(a_ctypes))]
        plen = int(rng.integers(40, 200))
        path[i] = "/" + "".join(chr(c) for c in rng.choice(np.frombuffer(b"abcdefABCDEF0123456789+/=", np.uint8), plen))
        hour[i] = int(rng.integers(1, 6))
        status[i] = 200
    minute = rng.integers(0, 60, n)
    sec = rng.integers(0, 60, n)
    ptime = [f"{h:02d}:{m:02d}:{s:02d}" for h, m, s in zip(hour, minute, sec)]
    client = ((10 << 24) | (2 << 16) | cli).astype(np.uint32)
    fulluri = [f"http://{h}{p}" for h, p in zip(host, path)]
    cols = {
        "p_date": StringColumn.from_list([date] * n), "p_time": StringColumn.from_list(ptime),
        "clientip": client, "host": StringColumn.from_list(host), "reqmethod": StringColumn.from_list(method),
        "useragent": StringColumn.from_list(ua), "resconttype": StringColumn.from_list(ctype),
        "duration": rng.integers(1, 5000, n).astype(np.int64), "username": StringColumn.from_list(["-"] * n),
        "authgroup": StringColumn.from_list(["-"] * n), "exceptionid": StringColumn.from_list(["-"] * n),
        "filterresult": StringColumn.from_list(["OBSERVED"] * n), "webcat": StringColumn.from_list(["-"] * n),
        "referer": StringColumn.from_list(["-"] * n), "respcode": status.astype(np.int32),
        "action": StringColumn.from_list(["TCP_NC_MISS"] * n), "urischeme": StringColumn.from_list(["http"] * n),
        "uriport": np.full(n, 80, np.int32), "uripath": StringColumn.from_list(path),
        "uriquery": StringColumn.from_list(["-"] * n), "uriextension": StringColumn.from_list(["html"] * n),
        "serverip": np.full(n, (93 << 24) | 1, np.uint32), "scbytes": rng.integers(200, 200000, n).astype(np.int64),
        "csbytes": rng.integers(100, 2000, n).astype(np.int64), "virusid": StringColumn.from_list(["-"] * n),
        "bcappname": StringColumn.from_list(["-"] * n), "bcappoperation": StringColumn.from_list(["-"] * n),
        "fulluri": StringColumn.from_list(fulluri),
    }
    labels[anomaly_rows] = -1
    return ProxyDay(cols=cols, anomaly_rows=anomaly_rows, labels=labels)


def write_log(day: ProxyDay, path: str) -> None:
    """Bluecoat main-format access log with a #Fields header."""
    from ..io.results import ip_str
    c = day.cols
    order = ["p_date", "p_time", "duration", "clientip", "username", "authgroup", "exceptionid", "filterresult",
             "webcat", "referer", "respcode", "action", "reqmethod", "resconttype", "urischeme", "host", "uriport",
             "uripath", "uriquery", "uriextension", "useragent", "serverip", "scbytes", "csbytes", "virusid"]
    with open(path, "w") as f:
        f.write("#Software: SGOS 6.5\n#Fields: " + " ".join(PROXY_FIELDS) + "\n")
        for i in range(day.n):
            vals = []
            for name in order:
                v = c[name]
                s = v[i] if isinstance(v, StringColumn) else (ip_str(v[i]) if name in ("clientip", "serverip") else str(v[i]))
                vals.append(f'"{s}"' if (" " in s or s == "") else s)
            f.write(" ".join(vals) + "\n")
