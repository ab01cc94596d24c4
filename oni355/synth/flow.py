"""Seeded synthetic netflow day with random-init topic priors and planted anomalies.

The reference shipped no data generator (it relied on real nfcapd sensors and the oni-demo
dataset); the north star asks for synthetic netflow "of the named shape
with random-init topic priors" (BASELINE.json). Generative model:

* ``n_profiles`` behaviour profiles (web browsing, DNS, mail, SSH admin, backups, P2P, ...), each a
  distribution over service port, hour of day, bytes and packets;
* every internal host (a document) has a profile mix θ* ~ Dir(alpha_true) (sparse);
* host activity is Zipf-distributed (a few hosts own most flows: NAT gateways, resolvers);
* each flow: profile z ~ θ*[src], server from the profile's pool, port/hour/bytes/packets from z;
* ``n_anomalies`` planted flows on hosts drawn by activity: an ordinary flow of a profile the host
  never uses, to that profile's server (lateral movement; see the comment at the plant) -- ground
  truth for "planted anomalies rank in the top-N" tests. ``anomaly_kind="rare-service"`` plants
  the round-1/2 rare-port flows to fresh external addresses instead (their ports are kept out of
  the realistic day's long tail).

Columns follow the flow schema of SURVEY.md §2.7 (nfdump CSV → Hive ``flow`` table).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

# (name, service ports, port weights, server-side?, peak hour, hour sd, log-bytes mu, sd, bytes/pkt)
_PROFILES = [
    ("web", [80, 443, 8080], [0.3, 0.65, 0.05], 10, 3.0, 8.5, 1.2, 700),
    ("dns", [53], [1.0], 12, 6.0, 5.0, 0.4, 90),
    ("mail", [25, 587, 993, 143], [0.4, 0.3, 0.2, 0.1], 9, 2.5, 9.5, 1.5, 900),
    ("ssh", [22], [1.0], 14, 3.0, 7.5, 1.8, 120),
    ("backup", [873, 445], [0.5, 0.5], 2, 1.0, 15.0, 1.0, 1400),
    ("p2p", [6881, 51413], [0.5, 0.5], 21, 2.0, 11.0, 2.0, 1100),
    ("ntp", [123], [1.0], 12, 7.0, 4.4, 0.1, 76),
    ("ldap", [389, 636, 88], [0.4, 0.3, 0.3], 8, 2.0, 7.0, 0.8, 300),
    ("db", [3306, 5432, 1433], [0.4, 0.4, 0.2], 11, 4.0, 10.0, 1.5, 1000),
    ("rdp", [3389], [1.0], 15, 2.5, 12.0, 1.2, 800),
    ("snmp", [161, 162], [0.8, 0.2], 12, 7.0, 5.5, 0.3, 150),
    ("smb", [445, 139], [0.8, 0.2], 13, 3.0, 10.5, 1.5, 1200),
    ("https-api", [443], [1.0], 3, 2.0, 6.5, 0.6, 400),
    ("video", [443, 1935], [0.7, 0.3], 20, 2.0, 16.0, 1.0, 1400),
    ("syslog", [514], [1.0], 12, 7.0, 6.0, 0.5, 200),
    ("proxy", [3128, 8080], [0.6, 0.4], 11, 3.0, 9.0, 1.3, 800),
    ("vpn", [500, 4500], [0.5, 0.5], 7, 2.0, 11.0, 1.5, 1000),
    ("dhcp", [67, 68], [0.5, 0.5], 8, 3.0, 5.8, 0.2, 330),
    ("ftp", [21, 20], [0.5, 0.5], 16, 2.0, 12.5, 1.5, 1400),
    ("monitoring", [9100, 5666], [0.5, 0.5], 12, 7.0, 7.2, 0.4, 500),
]

LT_REPEAT = 8  # realistic-vocabulary day: flows per (host, long-tail behaviour) pair
LT_MAX_SLOTS = 64  # ... and at most this many behaviours per host (a gateway repeats its own)

# rarely-used service ports (none is in a profile): planted anomalies draw from all of them so
# that each anomaly is an individually rare word, not one more frequent pattern
_ANOMALY_PORTS = [7, 9, 13, 19, 23, 37, 42, 69, 70, 79, 102, 111, 113, 119, 135, 137, 177, 179, 194, 201, 264,
                  318, 383, 427, 464, 497, 512, 513, 515, 520, 540, 554, 631, 646, 666, 749, 750, 902, 992, 1011]


@dataclass
class FlowDay:
    cols: dict            # column name -> numpy array (flow schema)
    theta_true: np.ndarray  # [n_hosts, n_profiles]
    host_ips: np.ndarray  # uint32 [n_hosts]
    anomaly_rows: np.ndarray  # int64 row ids of planted anomalies
    # generating label of every row (ground truth for tools/oracle_recall.py): the behaviour
    # profile p (0..n_profiles-1), n_profiles + b for long-tail behaviour b of the realistic day,
    # -1 for a planted anomaly
    labels: np.ndarray | None = None

    @property
    def n(self) -> int:
        return int(self.cols["sip"].shape[0])


def _ip(a, b, c, d):
    return (np.uint32(a) << np.uint32(24)) | (np.uint32(b) << np.uint32(16)) | (np.uint32(c) << np.uint32(8)) | np.uint32(d)


def ip_to_str(ip: int) -> str:
    ip = int(ip) & 0xFFFFFFFF
    return f"{ip >> 24}.{(ip >> 16) & 255}.{(ip >> 8) & 255}.{ip & 255}"


def str_to_ip(s: str) -> int:
    a, b, c, d = (int(x) for x in s.strip().split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def generate_flows(n: int, seed: int = 7, n_hosts: int | None = None, n_profiles: int = 20,
                   alpha_true: float = 0.08, zipf_a: float = 1.15, n_anomalies: int | None = None,
                   date=(2016, 7, 8), rank: int = 0, wide_vocab: bool = False, ipv6_frac: float = 0.0,
                   anomaly_hosts: str = "active", anomaly_kind: str = "rare-service",
                   support_min: float = 0.02, lt_codebook: float = 0.01) -> FlowDay:
    """Generate ``n`` flows. ``rank`` offsets the RNG stream (weak-scaling shards of one day).

    ``wide_vocab``: a realistic-vocabulary day (SURVEY.md §7.5 sizing, V ≈ 1e5–1e6 flow words):
    half of the flows repeat one of their host's long-tail behaviours (a service port
    anywhere in 1..1024 with its own hour, volume and server) instead of a profile flow, and 20 %
    of the flows are server-to-server (both ports low / both high), so every (port, time, bytes,
    packets, direction) bin fills. ``lt_codebook``: long-tail behaviours per flow (codebook size
    n · lt_codebook; 0.01 → V ≈ 1.7e5 flow words at 12.5M flows, 0.04 → V ≈ 4-5e5)."""
    rng = np.random.default_rng([seed, rank])
    n_profiles = min(n_profiles, len(_PROFILES))
    prof = _PROFILES[:n_profiles]
    if n_hosts is None:
        n_hosts = max(64, n // 25)
    if n_anomalies is None:
        n_anomalies = max(5, min(200, n // 50_000))
    # hosts: 10.x.y.z (shared across ranks: same hosts appear in every shard)
    hrng = np.random.default_rng([seed, 0xABCD])
    hid = np.arange(n_hosts, dtype=np.int64)
    host_ips = _ip(10, (hid >> 16) & 255, (hid >> 8) & 255, hid & 255).astype(np.uint32)
    theta = hrng.dirichlet(np.full(n_profiles, alpha_true), size=n_hosts)
    # support cut: a host never uses a profile of true weight < support_min (a Dirichlet draw has
    # no exact zeros, and its tails would make every busy host do a little of everything -- each
    # such flow an unplanted off-profile event)
    theta = np.where(theta >= support_min, theta, 0.0)
    top1 = np.argmax(theta, axis=1)
    theta[np.arange(n_hosts), top1] += (theta.sum(1) == 0)
    theta /= theta.sum(1, keepdims=True)
    # servers per profile: 172.16.<p>.<i>
    n_srv = max(4, min(250, n_hosts // 20))
    # host activity: Zipf over a random permutation of hosts
    w = 1.0 / np.power(np.arange(1, n_hosts + 1, dtype=np.float64), zipf_a)
    w = w[hrng.permutation(n_hosts)]
    w /= w.sum()
    src = rng.choice(n_hosts, size=n, p=w)
    # profile per flow: inverse-CDF on flattened cumulative rows
    cum = np.cumsum(theta, axis=1)
    cum[:, -1] = 1.0
    u = rng.random(n)
    flat = (cum + np.arange(n_hosts)[:, None]).ravel()
    z = np.searchsorted(flat, src + u, side="right") - src * n_profiles
    z = np.clip(z, 0, n_profiles - 1)
    labels = z.astype(np.int32)

    port_of = np.zeros(n, dtype=np.int64)
    hour_f = np.zeros(n)
    lbytes = np.zeros(n)
    bpp = np.zeros(n)
    for k, (_, ports, pw, peak, hsd, mu, sd, bp) in enumerate(prof):
        m = z == k
        cnt = int(m.sum())
        if not cnt:
            continue
        port_of[m] = rng.choice(ports, size=cnt, p=np.asarray(pw) / np.sum(pw))
        hour_f[m] = rng.normal(peak, hsd, size=cnt)
        lbytes[m] = rng.normal(mu, sd, size=cnt)
        bpp[m] = bp * np.exp(rng.normal(0, 0.2, size=cnt))
    srv = rng.integers(0, n_srv, size=n)
    dip = _ip(172, 16, z & 255, srv & 255).astype(np.uint32)
    if wide_vocab:
        # Half the flows come from a codebook of ~n/100 long-tail service behaviours (a well-known
        # port of the ~1k-port pool, an hour, a volume, a packet size and a server of its own):
        # the day's vocabulary grows to V ≈ 2e5-4e5 flow words at 12.5M flows (SURVEY.md §7.5
        # sizing: the q table leaves L2). Every host owns a few behaviours of the codebook
        # and its long-tail flows repeat them -- a backup agent, a licence server, a monitoring
        # probe recur from the same hosts to the same servers -- so a long-tail word is common in
        # the documents that carry it. Drawing behaviours uniformly over all hosts and the
        # profile servers instead scattered each over ~50 unrelated documents, where P(word |
        # doc) cannot tell them from a planted row (recall 0.245 at 12.5M flows,
        # profiles/r3/recall_sweep_codebook.jsonl). The anomalies' rare services are not in the pool.
        lt = np.nonzero(rng.random(n) < 0.5)[0]
        crng = np.random.default_rng([seed, 0xC0DE])
        W = max(1000, int(n * lt_codebook))
        pool = np.setdiff1d(np.arange(1, 1025), _ANOMALY_PORTS)
        cb_port = pool[crng.integers(0, pool.size, W)]
        cb_hour = crng.uniform(0.0, 24.0, W)
        cb_lbytes = crng.uniform(4.0, 18.0, W)
        cb_bpp = np.exp(crng.uniform(np.log(40.0), np.log(1500.0), W))
        n_lts = max(16, W // 8)  # long-tail servers 172.17-31.x.y, ~8 behaviours each
        cb_srv = crng.integers(0, n_lts, W)
        # each host owns ⌈(its long-tail flows) / LT_REPEAT⌉ behaviours, so every (host, behaviour)
        # pair recurs ~LT_REPEAT times in the host's document
        h_lt = src[lt]
        slots = np.clip(-(-np.bincount(h_lt, minlength=n_hosts) // LT_REPEAT), 1, LT_MAX_SLOTS)
        first = np.concatenate([[0], np.cumsum(slots)[:-1]])
        # slots deal the codebook out round-robin (shuffled): every behaviour has ~Σslots / W
        # owners, so none is a day-unique word
        orng = np.random.default_rng([seed, 0x0515])
        n_sl = int(slots.sum())
        own = np.concatenate([orng.permutation(W) for _ in range(-(-n_sl // W))])[:n_sl]
        own = own[orng.permutation(n_sl)]
        b = own[first[h_lt] + (rng.random(lt.size) * slots[h_lt]).astype(np.int64)]
        labels[lt] = n_profiles + b
        port_of[lt] = cb_port[b]
        hour_f[lt] = cb_hour[b]
        lbytes[lt] = cb_lbytes[b]
        bpp[lt] = cb_bpp[b]
        s = cb_srv[b]
        dip[lt] = _ip(172, 17 + (s >> 16), (s >> 8) & 255, s & 255)
    sip = host_ips[src]
    eph = rng.integers(1025, 65536, size=n)
    # ~15% of flows are recorded from the server side (service port in sport)
    flip = rng.random(n) < 0.15
    if wide_vocab:
        flip[lt] = False  # a long-tail behaviour is one word: always recorded client side
    sport = np.where(flip, port_of, eph)
    dport = np.where(flip, eph, port_of)
    if wide_vocab:
        s2s = rng.random(n) < 0.2  # server-to-server: both low (111111) or both high (333333)
        s2s[lt] = False
        both_low = s2s & (rng.random(n) < 0.5)
        both_high = s2s & ~both_low
        sport = np.where(both_low, rng.integers(1, 1025, size=n), np.where(both_high, rng.integers(1025, 65536, size=n), sport))
        dport = np.where(both_low, rng.integers(1, 1025, size=n), np.where(both_high, rng.integers(1025, 65536, size=n), dport))
    sip2 = np.where(flip, dip, sip)
    dip2 = np.where(flip, sip, dip)

    hour = np.mod(np.floor(hour_f), 24).astype(np.int64)
    minute = rng.integers(0, 60, size=n)
    if wide_vocab:
        minute[lt] = (cb_hour[b] * 60).astype(np.int64) % 60  # scheduled: one time bin per behaviour
    second = rng.integers(0, 60, size=n)
    ibyt = np.maximum(40, np.exp(lbytes)).astype(np.int64)
    ipkt = np.maximum(1, np.round(ibyt / np.maximum(bpp, 40))).astype(np.int64)

    # planted anomalies. anomaly_hosts "active" (default): the compromised hosts are drawn like any
    # flow's source (by activity); "quiet": the least active tenth of the hosts.
    #
    # anomaly_kind "offprofile" (default): the host makes an ordinary flow of the profile it is
    # least likely to use (θ*[host, p] = 0 after the support cut) to one of that profile's servers
    # -- a workstation reaching a database or backup server it never talks to (lateral
    # movement). What P(word | doc) scoring can rank: a token is scored with its own topic in the
    # counts, so a word that only the anomaly uses (a day-unique rare-service word) is sampled
    # into its host's dominant topic and scores like any on-profile flow of that host, while a
    # word that the profile's own hosts use often pulls the token into the profile's topic, where
    # the host has almost no mass: θ[host, B] ≈ (1 + α) / (n_host + Kα). The score falls with the
    # host's activity, so the anomaly is rare FOR A HOST WHOSE BEHAVIOUR IS KNOWN.
    # "rare-service": the round-1/2 plant -- a rare service port at an odd hour with outsized
    # volume to a fresh external address (203.0.113.0/24): individually unique words, which the
    # scoring above ranks no lower than any rare flow of a small document.
    anomaly_rows = np.sort(rng.choice(n, size=min(n_anomalies, n), replace=False))
    na = anomaly_rows.size
    labels[anomaly_rows] = -1
    if na:
        if anomaly_hosts == "quiet":
            quiet = np.argsort(w)[: max(1, n_hosts // 10)]
            a_src = quiet[rng.integers(0, quiet.size, size=na)]
        else:
            a_src = src[anomaly_rows]
        sip2[anomaly_rows] = host_ips[a_src]
        sport[anomaly_rows] = rng.integers(1025, 65536, size=na)
        if anomaly_kind == "rare-service":
            dip2[anomaly_rows] = _ip(203, 0, 113, rng.integers(1, 255, size=na) & 255)
            dport[anomaly_rows] = rng.choice(_ANOMALY_PORTS, size=na)
            hour[anomaly_rows] = rng.integers(1, 6, size=na)
            ibyt[anomaly_rows] = rng.integers(500_000_000, 900_000_000, size=na)
            # volume shape: a few giant packets, or a flood of them
            flood = rng.random(na) < 0.5
            ipkt[anomaly_rows] = np.where(flood, rng.integers(400_000, 600_000, size=na), rng.integers(1, 3, size=na))
        elif anomaly_kind == "offprofile":
            # the profile with the least true mass for the host; ties (several zeros after the
            # support cut) broken at random so the anomalies spread over profiles
            pert = theta[a_src] + rng.random((na, n_profiles)) * 1e-9
            p_off = np.argmin(pert, axis=1)
            dip2[anomaly_rows] = _ip(172, 16, p_off & 255, rng.integers(0, n_srv, size=na) & 255)
            for j, pk in enumerate(p_off.tolist()):
                _, ports, pw, peak, hsd, mu, sd, bp = prof[pk]
                r = anomaly_rows[j]
                dport[r] = ports[int(np.argmax(pw))]
                hour[r] = int(np.floor(rng.normal(peak, hsd))) % 24
                ibyt[r] = max(40, int(np.exp(rng.normal(mu, sd))))
                ipkt[r] = max(1, int(round(ibyt[r] / max(bp, 40))))
        else:
            raise ValueError(f"unknown anomaly_kind {anomaly_kind!r}")

    v6_rows = None
    if ipv6_frac > 0:
        v6_host = np.random.default_rng([seed, 0x6666]).random(n_hosts) < ipv6_frac
        v6_rows = v6_host[src]
        if na:
            v6_rows[anomaly_rows] = False

    y, mo, d = date
    unix = (np.int64(1467936000) + hour * 3600 + minute * 60 + second).astype(np.int64)
    cols = {
        "treceived": unix,
        "unix_tstamp": unix,
        "tryear": np.full(n, y, dtype=np.int32),
        "trmonth": np.full(n, mo, dtype=np.int32),
        "trday": np.full(n, d, dtype=np.int32),
        "trhour": hour.astype(np.int32),
        "trminute": minute.astype(np.int32),
        "trsec": second.astype(np.int32),
        "tdur": np.round(rng.exponential(2.0, size=n), 3).astype(np.float32),
        "sip": sip2.astype(np.uint32),
        "dip": dip2.astype(np.uint32),
        "sport": sport.astype(np.int32),
        "dport": dport.astype(np.int32),
        "proto": np.where(np.isin(port_of, [53, 123, 161, 162, 67, 68, 69, 514, 500, 4500]), 17, 6).astype(np.int32),
        "flag": np.zeros(n, dtype=np.int32),
        "fwd": np.zeros(n, dtype=np.int32),
        "stos": np.zeros(n, dtype=np.int32),
        "ipkt": ipkt,
        "ibyt": ibyt,
        "opkt": np.zeros(n, dtype=np.int64),
        "obyt": np.zeros(n, dtype=np.int64),
        "input": np.zeros(n, dtype=np.int32),
        "output": np.zeros(n, dtype=np.int32),
        "sas": np.zeros(n, dtype=np.int32),
        "das": np.zeros(n, dtype=np.int32),
        "dtos": np.zeros(n, dtype=np.int32),
        "dir": np.zeros(n, dtype=np.int32),
        "rip": np.zeros(n, dtype=np.uint32),
    }
    if v6_rows is not None and v6_rows.any():
        from ..store.columnar import StringColumn

        import ipaddress

        def v6_text(ip4: np.ndarray) -> list[str]:  # 2001:db8:<ip4 hi>:<ip4 lo>::1 in RFC 5952 form
            base = int(ipaddress.IPv6Address("2001:db8::1"))
            return [ipaddress.IPv6Address(base | (x << 64)).compressed for x in ip4.astype(np.int64).tolist()]

        idx = np.nonzero(v6_rows)[0]
        for k4, k6 in (("sip", "sip6"), ("dip", "dip6")):
            txt = [""] * n
            for i, t in zip(idx.tolist(), v6_text(cols[k4][idx])):
                txt[i] = t
            cols[k6] = StringColumn.from_list(txt)
            cols[k4] = np.where(v6_rows, 0, cols[k4]).astype(np.uint32)
    return FlowDay(cols=cols, theta_true=theta, host_ips=host_ips, anomaly_rows=anomaly_rows, labels=labels)


def generate_flows_sharded(per: int, parts: int, seed: int = 7, n_hosts: int | None = None, procs: int = 8,
                           **kw) -> FlowDay:
    """The ``parts`` weak-scaling shards (rank 0..parts-1, ``per`` flows each, one host population)
    of a ``per·parts``-flow day concatenated into ONE day -- e.g. all of a 1B-token day on one GPU
    -- generated by ``procs`` forked workers writing straight into shared-memory columns (a 500M-flow
    day is ~68 GB of columns and ~10 min of single-process generation). Row ids of the planted
    anomalies are offset by their shard's position."""
    import multiprocessing as mp
    from multiprocessing import shared_memory

    if n_hosts is None:
        n_hosts = max(64, per * parts // 25)
    probe = generate_flows(min(per, 1000), seed=seed, n_hosts=n_hosts, rank=0, **kw)
    if any(not isinstance(v, np.ndarray) for v in probe.cols.values()):
        raise ValueError("sharded generation supports numeric columns only (no IPv6 text columns)")
    n = per * parts
    shapes = dict(probe.cols, _labels=probe.labels)
    shm = {k: shared_memory.SharedMemory(create=True, size=max(1, n * v.dtype.itemsize))
           for k, v in shapes.items()}
    spec_ = {k: (s.name, shapes[k].dtype.str) for k, s in shm.items()}
    ctx = mp.get_context("fork")

    def work(r: int, q) -> None:
        d = generate_flows(per, seed=seed, n_hosts=n_hosts, rank=r, **kw)
        src = dict(d.cols, _labels=d.labels)
        for k, (name, dt) in spec_.items():
            s = shared_memory.SharedMemory(name=name)
            np.ndarray((n,), dtype=np.dtype(dt), buffer=s.buf)[r * per:(r + 1) * per] = src[k]
            s.close()
        q.put((r, d.anomaly_rows + r * per))

    q = ctx.Queue()
    anomalies = {}
    pending = list(range(parts))
    running: dict = {}
    try:
        while pending or running:
            while pending and len(running) < max(1, procs):
                r = pending.pop(0)
                running[r] = ctx.Process(target=work, args=(r, q))
                running[r].start()
            r, rows = q.get(timeout=3600)
            anomalies[r] = rows
            running.pop(r).join()
    finally:
        for p in running.values():
            p.terminate()
            p.join()
    cols = {}
    for k, s in shm.items():
        # own copy in this process's memory (plain numpy: pinning and the columnar store expect it),
        # then release the shared segment
        cols[k] = np.ndarray((n,), dtype=np.dtype(spec_[k][1]), buffer=s.buf).copy()
        s.close()
        s.unlink()
    labels = cols.pop("_labels")
    return FlowDay(cols=cols, theta_true=probe.theta_true, host_ips=probe.host_ips,
                   anomaly_rows=np.concatenate([anomalies[r] for r in range(parts)]), labels=labels)
