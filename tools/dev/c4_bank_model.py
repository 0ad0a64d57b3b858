"""Dev: LDS bank model of bp_ms_lds64_kernel's check-state accesses on the C4
graph, for a check -> state-slot permutation.  Per wave instruction (wave w,
owned-column round r, edge k) and 32-lane half: u64 state ops (m1 / m2 reads
and ds_min_u64) bank by slot mod 32, the b32 bit-word ops (parw / hdw / tiew)
by (slot >> 5) mod 32; reads cost the most distinct addresses on one bank,
atomics the most lanes on one bank (same-address RMWs serialise).  Prints the
model's cycles for the identity slots and for a greedy + annealed assignment."""
import os
import sys

import numpy as np
import scipy.sparse as sp

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
d = np.load(os.path.join(REPO, "tests", "golden", "hgp_80_3_4_s2025_checks.npz"))
H = sp.csr_matrix((np.ones(d["hz_indices"].size, np.uint8), d["hz_indices"], d["hz_indptr"]), shape=tuple(d["hz_shape"]))
m, n = H.shape
Hc = H.tocsc()
Hc.sort_indices()
T, VPT, DC = 1024, (n + 1023) // 1024, 4
halves = []  # arrays of checks per (w, r, k, half)
for w in range(T // 64):
    for r in range(VPT):
        for k in range(DC):
            for h in range(2):
                ch = []
                for l in range(32 * h, 32 * h + 32):
                    t = 64 * w + l
                    j = r * T + (67 * t) % T
                    if j < n:
                        rows = Hc.indices[Hc.indptr[j]:Hc.indptr[j + 1]]
                        if k < rows.size:
                            ch.append(rows[k])
                if ch:
                    halves.append(np.array(ch))
print(f"m={m} n={n} halves={len(halves)}")
W_U64R, W_U64A, W_B32R, W_B32A = 3.0, 2.0, 1.0, 0.5


def cost_half(s):
    c = 0.0
    key = s % 32
    # u64 reads: distinct addresses per bank; atomics: lanes per bank
    u, inv = np.unique(s, return_inverse=True)
    c += W_U64R * np.bincount(u % 32, minlength=32).max()
    c += W_U64A * np.bincount(key, minlength=32).max()
    wd = s >> 5
    uw = np.unique(wd)
    c += W_B32R * np.bincount(uw % 32, minlength=32).max()
    c += W_B32A * np.bincount(wd % 32, minlength=32).max()
    return c


def total(slot):
    return sum(cost_half(slot[hh]) for hh in halves)


ideal = len(halves) * (W_U64R + W_U64A + W_B32R + W_B32A)
ident = np.arange(m)
print("identity", total(ident), "ideal", ideal)
rng = np.random.default_rng(0)
print("random", total(rng.permutation(m)))
