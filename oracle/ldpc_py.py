"""Pure-Python restatement of ldpc v1's BP loops (test infrastructure only).

A second, independent transcription of the published ldpc v1 ``bp_decoder``
routines (quantumgizmos/ldpc rev 7909a97d; see oracle/qdec_oracle.h), written as
plain Python loops over a mod2sparse-like edge list.  Python floats are IEEE
doubles and ``math.log`` is the platform libm, so on small cases this must agree
bit for bit with the C oracle's fp64 mode.  Too slow for anything but tiny
shot counts -- it exists only to cross-check oracle/qdec_oracle.c.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse as sp


class _Graph:
    def __init__(self, H):
        H = sp.csr_matrix(H)
        H.sort_indices()
        self.m, self.n = H.shape
        self.rows = [list(range(H.indptr[i], H.indptr[i + 1])) for i in range(self.m)]
        self.col_of = [int(c) for c in H.indices]
        self.row_of = [i for i in range(self.m) for _ in range(H.indptr[i], H.indptr[i + 1])]
        self.cols = [[] for _ in range(self.n)]
        for i in range(self.m):
            for e in self.rows[i]:
                self.cols[self.col_of[e]].append(e)


def bp_decode(H, probs, syndrome, *, method="ms", max_iter=0, ms_scaling=0.0):
    """Returns (decoding uint8[n], log_prob_ratios float[n], iter, converge).

    Arithmetic is numpy float64 scalar arithmetic, i.e. C semantics (x/0 -> inf,
    0*inf -> nan) as in ldpc's compiled loops."""
    with np.errstate(all="ignore"):
        return _bp_decode(H, probs, syndrome, method=method, max_iter=max_iter, ms_scaling=ms_scaling)


def _bp_decode(H, probs, syndrome, *, method, max_iter, ms_scaling):
    g = _Graph(H)
    m, n = g.m, g.n
    probs = [np.float64(v) for v in np.broadcast_to(np.asarray(probs, dtype=float), (n,))]
    s = [int(v) & 1 for v in syndrome]
    if max_iter <= 0:
        max_iter = n
    E = len(g.col_of)
    b2c = [0.0] * E
    c2b = [0.0] * E
    sgn = [0] * E
    x = [0] * n
    lpr = [0.0] * n
    if method == "ms":
        for j in range(n):
            for e in g.cols[j]:
                b2c[e] = math.log((1 - probs[j]) / probs[j])
    else:
        for j in range(n):
            for e in g.cols[j]:
                b2c[e] = probs[j] / (1 - probs[j])
    it = 0
    for it in range(1, max_iter + 1):
        if method == "ms":
            alpha = 1.0 - 2.0 ** (-it) if ms_scaling == 0 else ms_scaling
            for i in range(m):
                temp, sg = 1e308, s[i]
                for e in g.rows[i]:
                    c2b[e] = temp
                    sgn[e] = sg
                    if abs(b2c[e]) < temp:
                        temp = abs(b2c[e])
                    if b2c[e] <= 0:
                        sg = 1 - sg
                temp, sg = 1e308, 0
                for e in reversed(g.rows[i]):
                    if temp < c2b[e]:
                        c2b[e] = temp
                    sgn[e] += sg
                    c2b[e] *= ((-1) ** sgn[e]) * alpha
                    if abs(b2c[e]) < temp:
                        temp = abs(b2c[e])
                    if b2c[e] <= 0:
                        sg = 1 - sg
            for j in range(n):
                temp = math.log((1 - probs[j]) / probs[j])
                for e in g.cols[j]:
                    b2c[e] = temp
                    temp += c2b[e]
                lpr[j] = temp
                x[j] = 1 if temp <= 0 else 0
                temp = 0.0
                for e in reversed(g.cols[j]):
                    b2c[e] += temp
                    temp += c2b[e]
        else:
            for i in range(m):
                temp = (-1.0) ** s[i]
                for e in g.rows[i]:
                    c2b[e] = temp
                    temp *= 2 / (1 + b2c[e]) - 1
                temp = 1.0
                for e in reversed(g.rows[i]):
                    c2b[e] *= temp
                    c2b[e] = (1 - c2b[e]) / (1 + c2b[e])
                    temp *= 2 / (1 + b2c[e]) - 1
            for j in range(n):
                temp = probs[j] / (1 - probs[j])
                for e in g.cols[j]:
                    b2c[e] = temp
                    temp *= c2b[e]
                    if math.isnan(temp):
                        temp = 1.0
                inv = np.float64(1.0) / np.float64(temp)
                lpr[j] = math.log(inv) if inv > 0 else (-math.inf if inv == 0 else math.nan)
                x[j] = 1 if temp >= 1 else 0
                temp = 1.0
                for e in reversed(g.cols[j]):
                    b2c[e] *= temp
                    temp *= c2b[e]
                    if math.isnan(temp):
                        temp = 1.0
        ok = True
        for i in range(m):
            p = 0
            for e in g.rows[i]:
                p ^= x[g.col_of[e]]
            if p != s[i]:
                ok = False
                break
        if ok:
            return np.array(x, np.uint8), np.array(lpr), it, 1
    return np.array(x, np.uint8), np.array(lpr), it, 0
