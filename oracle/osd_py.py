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


def _reduce(Hs):
    """Greedy pivot columns of Hs and a row transform T with (T Hs)[:r, piv] = I,
    so the solution over piv of Hs[:, piv] x = s is (T s)[:r] for every s."""
    m, n = Hs.shape
    A = np.concatenate([Hs % 2, np.eye(m, dtype=np.uint8)], axis=1).astype(np.uint8)
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
    return piv, A[:, n:]


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
    if not cands:
        return osd0, best
    # every candidate's pivot solution from one row transform of Hs[:, piv]
    # (full column rank), in candidate order; strict improvement keeps the earlier
    piv2, T = _reduce(Hs[:, piv])
    assert piv2 == list(range(len(piv)))
    r = len(piv)
    S2 = np.repeat(s[:, None], len(cands), axis=1).astype(np.int64)
    for ci, g in enumerate(cands):
        S2[:, ci] += Hs[:, g].astype(np.int64).sum(axis=1)
    XP = (T.astype(np.int64) @ (S2 % 2)) % 2
    for ci, g in enumerate(cands):
        w = int(XP[:r, ci].sum()) + len(g)
        if w < best_w:
            best, best_w = assemble(XP[:r, ci].astype(np.uint8), g), w
    return osd0, best
