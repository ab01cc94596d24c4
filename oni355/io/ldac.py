"""lda-c file formats (Blei's lda-c as forked by oni-lda-c; SURVEY.md §2.7, [U-H]).

* ``model.dat``            corpus: one line per document, ``M w1:c1 w2:c2 ...`` (0-based ids)
* ``<prefix>.beta``        K lines × V floats: log p(w | k)
* ``<prefix>.gamma``       D lines × K floats (VEM: variational Dirichlet; Gibbs: n_dk + α)
* ``<prefix>.other``       ``num_topics K`` / ``num_terms V`` / ``alpha a``
* ``likelihood.dat``       one line per iteration: ``<likelihood>\\t<convergence>``
* ``word-assignments.dat`` per document ``M w:z ...`` (Gibbs: one entry per token)

The C++ VEM engine (``oni355/_lib/bin/lda``) reads/writes the same files, so corpora and models
round-trip between the GPU sampler, the CPU engine and the reference's own tooling.
"""
from __future__ import annotations

import os

import numpy as np


def write_corpus(path: str, pair_doc, pair_word, pair_cnt, D: int) -> None:
    pair_doc = np.asarray(pair_doc, dtype=np.int64)
    pair_word = np.asarray(pair_word, dtype=np.int64)
    pair_cnt = np.asarray(pair_cnt, dtype=np.int64)
    ptr = np.searchsorted(pair_doc, np.arange(D + 1))
    with open(path, "w") as f:
        for d in range(D):
            lo, hi = ptr[d], ptr[d + 1]
            items = " ".join(f"{w}:{c}" for w, c in zip(pair_word[lo:hi], pair_cnt[lo:hi]))
            f.write(f"{hi - lo}{' ' if items else ''}{items}\n")


def read_corpus(path: str) -> list[tuple[np.ndarray, np.ndarray]]:
    docs = []
    with open(path) as f:
        for line in f:
            t = line.split()
            if not t:
                continue
            m = int(t[0])
            ws = np.array([int(x.split(":")[0]) for x in t[1:1 + m]], dtype=np.int64)
            cs = np.array([int(x.split(":")[1]) for x in t[1:1 + m]], dtype=np.int64)
            docs.append((ws, cs))
    return docs


def write_matrix(path: str, m: np.ndarray, fmt: str = "%5.10f") -> None:
    np.savetxt(path, np.asarray(m, dtype=np.float64), fmt=fmt, delimiter=" ")


def read_matrix(path: str) -> np.ndarray:
    return np.loadtxt(path, dtype=np.float64, ndmin=2)


def write_other(path: str, K: int, V: int, alpha: float) -> None:
    with open(path, "w") as f:
        f.write(f"num_topics {K}\nnum_terms {V}\nalpha {alpha:5.10f}\n")


def read_other(path: str) -> dict:
    out = {}
    with open(path) as f:
        for line in f:
            k, v = line.split()
            out[k] = float(v) if k == "alpha" else int(v)
    return out


def write_model(directory: str, prefix: str, log_beta: np.ndarray, gamma: np.ndarray, alpha: float) -> None:
    """log_beta: [K, V]; gamma: [D, K]."""
    os.makedirs(directory, exist_ok=True)
    write_matrix(os.path.join(directory, f"{prefix}.beta"), log_beta)
    write_matrix(os.path.join(directory, f"{prefix}.gamma"), gamma)
    write_other(os.path.join(directory, f"{prefix}.other"), log_beta.shape[0], log_beta.shape[1], alpha)


def write_likelihood(path: str, lls: list[tuple[int, float]]) -> None:
    with open(path, "w") as f:
        prev = None
        for _, ll in lls:
            conv = 0.0 if prev is None or prev == 0 else (prev - ll) / prev
            f.write(f"{ll:10.10f}\t{conv:5.5e}\n")
            prev = ll


def write_word_assignments(path: str, doc_tok_ptr, tok_word, tok_z) -> None:
    ptr = np.asarray(doc_tok_ptr, dtype=np.int64)
    tw = np.asarray(tok_word)
    tz = np.asarray(tok_z)
    with open(path, "w") as f:
        for d in range(ptr.size - 1):
            lo, hi = ptr[d], ptr[d + 1]
            f.write(f"{hi - lo:04d}" + "".join(f" {w:04d}:{z:02d}" for w, z in zip(tw[lo:hi], tz[lo:hi])) + "\n")


def export_gibbs(directory: str, model, prefix: str = "final", word_assignments: bool = False) -> None:
    """Emit lda-c compatible files for a trained :class:`oni355.models.gibbs.GibbsLDA` (local docs)."""
    import torch

    from ..models.corpus import canonical_tokens
    K = model.K
    phi = model.phi()[:, :K].double().cpu().numpy()  # [V, K]
    gamma = (model.ndk_cur[: model.c.D_own, :K].double() + model.alpha).cpu().numpy()
    write_model(directory, prefix, np.log(phi.T), gamma, model.alpha)
    if model.likelihoods:
        write_likelihood(os.path.join(directory, "likelihood.dat"), model.likelihoods)
    if word_assignments:
        _, tword = canonical_tokens(model.c)
        write_word_assignments(os.path.join(directory, "word-assignments.dat"), model.c.doc_tok_ptr.cpu().numpy(),
                               tword.cpu().numpy(), model.canonical_z().cpu().numpy())
    _ = torch
