"""Checkpoint / resume for the Gibbs sampler.

A checkpoint is the topic assignment of every token (1 byte each) grouped by document key, plus
the sweep counter and the run's identity (K, α, β, seed, V, T). Every count table is recomputed
from z on restore, and the counter RNG makes the resumed chain bitwise identical to an
uninterrupted one. Shards are keyed by document, so a run may resume on a different GPU count
(documents are re-routed to their new owners).

Layout: ``<dir>/ckpt_s<sweep>_r<rank>of<world>.pt`` (+ ``manifest.json`` written by rank 0 after
all shards of a sweep are on disk; atomic renames throughout). lda-c-style ``NNN.*`` snapshots
are emitted separately by :mod:`oni355.io.ldac`.
"""
from __future__ import annotations

import glob
import json
import os

import torch


class Checkpointer:
    def __init__(self, directory: str, every: int = 0, comm=None, keep: int = 2):
        self.dir = directory
        self.every = int(every)
        self.comm = comm
        self.keep = keep
        os.makedirs(directory, exist_ok=True)

    @property
    def rank(self) -> int:
        return self.comm.rank if self.comm else 0

    @property
    def world(self) -> int:
        return self.comm.world if self.comm else 1

    def _ident(self, model) -> dict:
        """What the chain is a function of: a checkpoint resumes only a run of the same identity.
        ``chain`` names the sampler family and, for MH runs, the dense burn-in length (the MH
        chain and the dense chain are different Markov chains over the same z)."""
        ident = {"K": model.K, "alpha": model.alpha, "beta": model.beta, "seed": int(model.cfg.seed), "V": model.V}
        chain = getattr(model, "chain", None)
        if chain is not None:
            ident["chain"] = dict(chain)
        return ident

    def manifest(self) -> dict | None:
        p = os.path.join(self.dir, "manifest.json")
        if not os.path.exists(p):
            return None
        with open(p) as f:
            return json.load(f)

    def exists(self) -> bool:
        return self.manifest() is not None

    def save(self, model) -> str:
        c = model.c
        z = model.canonical_z().cpu()
        payload = {
            "ident": self._ident(model),
            "sweep": int(model.sweeps_done),
            "doc_keys": c.doc_keys.cpu(),
            "doc_tok_ptr": c.doc_tok_ptr.cpu(),
            # canonical position of each row's first token: non-zero only for pieces of documents
            # cut across ranks (pipeline.common.SplitPlan)
            "doc_pos0": _pos0(c).cpu(),
            "z": z,
            "likelihoods": list(model.likelihoods),
        }
        avg = model.average_state() if hasattr(model, "average_state") else None
        if avg is not None:
            # inside the posterior-averaging window: the samples so far; the doc-topic sums are
            # rows aligned with doc_keys, so a resume on another world size re-keys them
            payload["avg"] = avg
        name = f"ckpt_s{model.sweeps_done}_r{self.rank}of{self.world}.pt"
        path = os.path.join(self.dir, name)
        torch.save(payload, path + ".tmp")
        os.replace(path + ".tmp", path)
        if self.comm is not None:
            self.comm.barrier()
        if self.rank == 0:
            man = {"sweep": int(model.sweeps_done), "world": self.world, "ident": self._ident(model)}
            mp = os.path.join(self.dir, "manifest.json")
            with open(mp + ".tmp", "w") as f:
                json.dump(man, f)
            os.replace(mp + ".tmp", mp)
            self._gc(model.sweeps_done)
        if self.comm is not None:
            self.comm.barrier()
        return path

    def _gc(self, latest: int) -> None:
        sweeps = sorted({int(os.path.basename(p).split("_")[1][1:]) for p in glob.glob(os.path.join(self.dir, "ckpt_s*"))})
        for s in sweeps[: max(0, len(sweeps) - self.keep)]:
            if s == latest:
                continue
            for p in glob.glob(os.path.join(self.dir, f"ckpt_s{s}_r*")):
                os.remove(p)

    @staticmethod
    def _split_keys(keys: torch.Tensor, pos0: torch.Tensor) -> torch.Tensor:
        """Keys that are not one whole document in one row: pieces (pos0 > 0) or repeated keys."""
        u, cnt = torch.unique(keys, return_counts=True)
        return torch.unique(torch.cat([keys[pos0 > 0], u[cnt > 1]]))

    def restore(self, model) -> int:
        man = self.manifest()
        if man is None:
            raise FileNotFoundError(f"no checkpoint manifest in {self.dir}")
        if not _same_chain(man["ident"], self._ident(model), int(man["sweep"])):
            raise ValueError(f"checkpoint identity {man['ident']} != run {self._ident(model)} (a checkpoint resumes "
                             "only the chain that wrote it: same K, α, β, seed, vocabulary, sampler and MH burn-in)")
        sweep = int(man["sweep"])
        c = model.c
        mask = 0xFFFFFFFF
        my_keys = c.doc_keys.cpu().to(torch.int64) & mask
        my_ptr = c.doc_tok_ptr.cpu().to(torch.int64)
        my_len = my_ptr[1:] - my_ptr[:-1]
        my_pos0 = _pos0(c).cpu()
        z = torch.zeros(int(my_ptr[-1]) if my_ptr.numel() else 0, dtype=torch.uint8)
        found = torch.zeros(my_keys.numel(), dtype=torch.bool)
        # documents cut into pieces (here or in the checkpoint's run): whole-document z is
        # assembled from every shard's pieces, then sliced to this rank's ranges
        my_split = torch.unique(torch.cat([self._split_keys(my_keys, my_pos0), my_keys[my_len == 0]]))
        pieces: dict = {}
        # vectorised: every shard's documents are matched to this rank's by key (searchsorted) and
        # their token ranges copied with one index gather; shards holding none of them are skipped
        for p in sorted(glob.glob(os.path.join(self.dir, f"ckpt_s{sweep}_r*of{man['world']}.pt"))):
            d = torch.load(p, weights_only=True)
            if "likelihoods" in d and not model.likelihoods:
                model.likelihoods = [tuple(x) for x in d["likelihoods"]]
            keys = d["doc_keys"].to(torch.int64) & mask
            if keys.numel() == 0 or my_keys.numel() == 0:
                continue
            ptr = d["doc_tok_ptr"].to(torch.int64)
            pos0 = d.get("doc_pos0", torch.zeros(keys.numel(), dtype=torch.int64)).to(torch.int64)
            sk_split = torch.unique(torch.cat([self._split_keys(keys, pos0), my_split]))
            if sk_split.numel():
                isp = torch.isin(keys, sk_split)
                for r in torch.nonzero(isp).flatten().tolist():
                    ln = int(ptr[r + 1] - ptr[r])
                    if ln:
                        pieces.setdefault(int(keys[r]), []).append((int(pos0[r]), d["z"][int(ptr[r]):int(ptr[r]) + ln]))
                keep = ~isp
                keys, ptr_lo, ptr_hi = keys[keep], ptr[:-1][keep], ptr[1:][keep]
                if keys.numel() == 0:
                    continue
                ptr = None
            else:
                ptr_lo, ptr_hi = ptr[:-1], ptr[1:]
            order = torch.argsort(keys)
            sk = keys[order]
            pos = torch.searchsorted(sk, my_keys).clamp_(max=sk.numel() - 1)
            hit = sk[pos] == my_keys
            if not bool(hit.any()):
                continue
            dst = torch.nonzero(hit).flatten()
            src = order[pos[dst]]
            lens = ptr_hi[src] - ptr_lo[src]
            if not torch.equal(lens, my_len[dst]):
                bad = dst[torch.nonzero(lens != my_len[dst]).flatten()[0]]
                raise ValueError(f"checkpoint does not match corpus (doc key {int(my_keys[bad])})")
            n = int(lens.sum())
            rep = torch.repeat_interleave(torch.arange(dst.numel()), lens)
            within = torch.arange(n) - torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens)
            z[my_ptr[dst][rep] + within] = d["z"][ptr_lo[src][rep] + within]
            found[dst] = True
        for r in torch.nonzero(~found).flatten().tolist():
            ln = int(my_len[r])
            k = int(my_keys[r])
            if ln == 0:  # a split document's primary row: θ only, no tokens here
                found[r] = True
                continue
            if k not in pieces:
                continue
            full_len = max(p + int(v.numel()) for p, v in pieces[k])
            whole = torch.zeros(full_len, dtype=torch.uint8)
            cov = torch.zeros(full_len, dtype=torch.bool)
            for p, v in pieces[k]:
                whole[p:p + v.numel()] = v
                cov[p:p + v.numel()] = True
            p0 = int(my_pos0[r])
            if p0 + ln <= full_len and bool(cov[p0:p0 + ln].all()):
                z[int(my_ptr[r]):int(my_ptr[r]) + ln] = whole[p0:p0 + ln]
                found[r] = True
        if not bool(found.all()):
            miss = int(my_keys[torch.nonzero(~found).flatten()[0]])
            raise ValueError(f"checkpoint does not match corpus (doc key {miss} missing)")
        model.load_canonical_z(z, sweep)
        win = model.average_window if hasattr(model, "average_window") else None
        if win is not None and sweep >= win[0]:
            self._restore_average(model, sweep, man, win)
        return sweep


    def _restore_average(self, model, sweep: int, man: dict, win) -> None:
        """Resume inside the posterior-averaging window on ANY world size: the word-topic and topic
        sums are global (every shard holds the same), the doc-topic sums are matched to this
        rank's rows by document key (every row of a document cut into pieces carries the whole
        document's counts, so any of them serves)."""
        keys_all, dk_all, glob_avg = [], [], None
        for p in sorted(glob.glob(os.path.join(self.dir, f"ckpt_s{sweep}_r*of{man['world']}.pt"))):
            d = torch.load(p, weights_only=True)
            if "avg" not in d:
                raise ValueError(f"checkpoint shard {os.path.basename(p)} at sweep {sweep} lacks the posterior "
                                 f"samples of the averaging window {win}")
            if glob_avg is None:
                glob_avg = d["avg"]
            keys_all.append(d["doc_keys"].to(torch.int64) & 0xFFFFFFFF)
            dk_all.append(d["avg"]["dk"][: d["doc_keys"].numel()])
        if glob_avg is None:
            raise ValueError(f"no checkpoint shards at sweep {sweep}")
        keys = torch.cat(keys_all)
        dk = torch.cat(dk_all)
        my_keys = model.c.doc_keys.cpu().to(torch.int64) & 0xFFFFFFFF
        out = torch.zeros((max(my_keys.numel(), 1), dk.shape[1]), dtype=dk.dtype)
        if my_keys.numel():
            order = torch.argsort(keys, stable=True)
            sk = keys[order]
            pos = torch.searchsorted(sk, my_keys).clamp_(max=max(sk.numel() - 1, 0))
            hit = sk[pos] == my_keys if sk.numel() else torch.zeros_like(my_keys, dtype=torch.bool)
            if not bool(hit.all()):
                miss = int(my_keys[torch.nonzero(~hit).flatten()[0]])
                raise ValueError(f"averaging samples do not match the corpus (doc key {miss} missing)")
            out[: my_keys.numel()] = dk[order[pos]]
        model.load_average_state({"n": glob_avg["n"], "wk": glob_avg["wk"], "k": glob_avg["k"], "dk": out})

def _same_chain(saved: dict, run: dict, sweep: int) -> bool:
    """Does a checkpoint of identity ``saved`` at ``sweep`` lie on the chain ``run`` samples? Equal
    identities do; an MH run's state inside its dense burn-in is also a prefix of any MH run whose
    burn-in reaches that sweep (a 2-sweep run capped the same ONI_MH_BURN = 3 at 2)."""
    s, r = dict(saved), dict(run)
    # a manifest written before identities carried the chain holds the dense sampler's chain
    dense = {"sampler": "dense", "mh_burn": 0}
    sc, rc = s.pop("chain", None) or dense, r.pop("chain", None) or dense
    if s != r:
        return False
    if sc == rc:
        return True
    return sc.get("sampler") == rc.get("sampler") and sweep <= min(sc.get("mh_burn", 0), rc.get("mh_burn", 0))


def _pos0(c) -> torch.Tensor:
    """Canonical position of each corpus row's first token (0 unless the row is a piece)."""
    if c.split is not None and "doc_pos0" in c.split:
        return c.split["doc_pos0"].to(torch.int64)
    return torch.zeros(c.D, dtype=torch.int64)
