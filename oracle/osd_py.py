"""Dense numpy restatement of the OSD stage (test infrastructure only).

Same spec as exp_ldpc_amd/csrc/qdec_osd.cpp (this build's restatement of ldpc
v1's published OSD-0 / OSD-E / OSD-CS; ldpc itself is absent, so parity against
it is unpinned), written independently: column order by a stable argsort of the
BP log-probability ratios, plain row reduction on a dense uint8 matrix, and
candidates solved from scratch (no transform reuse).  Small cases only.
"""
from __future__ import annotations

import itertools

import numpy as np
import scipy.sparse as sp


def _solve_pivots(Hs, s):
    """Greedy pivot columns of Hs (column order as given) and the solution of
    Hs[:, piv] x = s; returns (piv list, x over piv)."""
    A = np.concatenate([Hs % 2, (s % 2)[:, None]], axis=1).astype(np.uint8)
    m, n = Hs.shape
    piv = []
    r = 0
    for c in range(n):
        if r >= m:
            break
        rows = np.nonzero(A[r:, c])[0]
        if rows.size == 0:
            continue
        p = r + rows[0]
        A[[r, p]] = A[[p, r]]
        mask = A[:, c].astype(bool)
        mask[r] = False
        A[mask] ^= A[r]
        piv.append(c)
        r += 1
    return piv, A[:r, n]


def osd_decode(H, syndrome, llr, method="osd_cs", order=0):
    """Returns (osd0, osdw) uint8[n]."""
    H = sp.csr_matrix(H).toarray() % 2
    m, n = H.shape
    cols = np.argsort(np.asarray(llr, dtype=np.float64), kind="stable")
    Hs = H[:, cols]
    s = np.asarray(syndrome, dtype=np.uint8) % 2
    piv, x0p = _solve_pivots(Hs, s)
    nonpiv = [c for c in range(n) if c not in set(piv)]

    def assemble(xp, g):
        xs = np.zeros(n, np.uint8)
        xs[piv] = xp
        for c in g:
            xs[c] ^= 1
        out = np.zeros(n, np.uint8)
        out[cols] = xs
        return out

    osd0 = assemble(x0p, [])
    if method == "osd0":
        return osd0, osd0.copy()
    best = osd0
    best_w = int(osd0.sum())
    lam = min(order, len(nonpiv))
    if method == "osd_e":
        cands = []
        for mask in range(1, 1 << lam):
            cands.append([nonpiv[t] for t in range(lam) if (mask >> t) & 1])
    else:
        cands = [[c] for c in nonpiv] + [[nonpiv[a], nonpiv[b]] for a, b in itertools.combinations(range(lam), 2)]
    for g in cands:
        s2 = (s + Hs[:, g].sum(axis=1)) % 2
        _, xp = _solve_pivots(Hs[:, piv], s2)  # same pivot set: full column rank
        cand = assemble(xp, g)
        w = int(cand.sum())
        if w < best_w:
            best, best_w = cand, w
    return osd0, best
