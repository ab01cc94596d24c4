"""CPU variational-EM LDA (oni-lda-c equivalent) -- ctypes wrapper of the C++ engine.

The reference-equivalent CPU path (BASELINE config 1: "10k-doc synthetic netflow corpus, 20-topic
LDA via oni-lda-c on CPU"). The same engine is available as the standalone ``lda`` CLI
(``oni355/_lib/bin/lda est|inf``) with lda-c file formats.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ..ops import native

native.register("oni_vem_est", [
    C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int, C.c_int, C.c_double,
    C.c_int, C.c_double, C.c_uint64, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
])


@dataclass
class VemResult:
    log_beta: np.ndarray  # [K, V]
    gamma: np.ndarray     # [D, K]
    alpha: float
    likelihood: np.ndarray
    iterations: int

    def theta(self) -> np.ndarray:
        return self.gamma / self.gamma.sum(1, keepdims=True)

    def phi(self) -> np.ndarray:
        """[V, K] p(w | k)."""
        return np.exp(self.log_beta).T.copy()


def estimate(doc_ptr, words, counts, V: int, K: int, alpha: float = 2.5, estimate_alpha: bool = True,
             var_max_iter: int = 20, var_convergence: float = 1e-6, em_max_iter: int = 100,
             em_convergence: float = 1e-4, seed: int = 4357, seeded: bool = False, threads: int = 0) -> VemResult:
    doc_ptr = np.ascontiguousarray(doc_ptr, dtype=np.int64)
    words = np.ascontiguousarray(words, dtype=np.int32)
    counts = np.ascontiguousarray(counts, dtype=np.int32)
    D = doc_ptr.size - 1
    if words.size != doc_ptr[-1] or counts.size != words.size:
        raise ValueError("doc_ptr / words / counts mismatch")
    if words.size and (words.min() < 0 or words.max() >= V):
        raise ValueError("word id out of range")
    log_beta = np.zeros((K, V), dtype=np.float64)
    gamma = np.zeros((D, K), dtype=np.float64)
    a_out = np.zeros(1, dtype=np.float64)
    lik = np.zeros(em_max_iter + 2, dtype=np.float64)
    iters = np.zeros(1, dtype=np.int32)
    rc = native.lib().oni_vem_est(doc_ptr.ctypes.data, words.ctypes.data, counts.ctypes.data, D, V, K, float(alpha),
                                  int(estimate_alpha), var_max_iter, var_convergence, em_max_iter, em_convergence,
                                  seed, int(seeded), threads, log_beta.ctypes.data, gamma.ctypes.data,
                                  a_out.ctypes.data, lik.ctypes.data, iters.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"oni_vem_est failed ({rc})")
    n = int(iters[0])
    return VemResult(log_beta, gamma, float(a_out[0]), lik[: min(n, lik.size)], n)
