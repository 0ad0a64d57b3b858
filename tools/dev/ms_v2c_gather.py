"""Dev: feasibility of a variable-major v2c layout for bp_ms_wave_kernel<double>.

Variables write their v2c messages lane-linearly (element (rv*4 + k)*64 +
(lane + rot[rv][k]) % 64: ds_write_b64, conflict-free); check lanes gather
their DRC messages with ds_read_b64 (2 groups of 32 lanes, class = element
% 32).  The check's read order is free (min / sign are order-independent).
Anneal over rot, the variable lane permutation inside degree classes and the
per-check read order; report LDS-array cycles of the check gathers.
"""
import os
import random
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "tests"))
from conftest import load_checks  # noqa: E402

rnd = random.Random(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
_, H = load_checks("hgp_12_3_4_s1234")
H = H.tocsr()
H.sort_indices()
m, n = H.shape
rp, ci = H.indptr, H.indices
Hc = H.tocsc()
Hc.sort_indices()
cdeg = np.diff(Hc.indptr)
DRC = int(np.diff(rp).max())
order = sorted(range(n), key=lambda j: cdeg[j])
slot_of = np.empty(n, int)
for s, j in enumerate(order):
    slot_of[j] = s
# edge -> (rv, k) of its variable
kpos = {}
for j in range(n):
    for k, i in enumerate(Hc.indices[Hc.indptr[j]:Hc.indptr[j + 1]]):
        kpos[(i, j)] = k
rot = [[0] * 4 for _ in range(4)]
# checks: edges as (variable)
edges = [list(ci[rp[i]:rp[i + 1]]) for i in range(m)]
# read order: perm per check over DRC slots (slot >= deg -> Big)
BIG = -1


def cls(i, t):
    j = rd[i][t]
    if j == BIG:
        return BIG
    s = slot_of[j]
    rv, lane = s // 64, s % 64
    return (lane + rot[rv][kpos[(i, j)]]) % 32


rd = [edges[i] + [BIG] * (DRC - len(edges[i])) for i in range(m)]


def groups_of(i):
    return i // 32  # 32-lane group index (rc*2 + half)


NGRP = (m + 31) // 32


def gcost(gidx, t):
    cnt = {}
    mx = 0
    for i in range(gidx * 32, min(m, gidx * 32 + 32)):
        c = cls(i, t)
        if c == BIG:
            continue
        cnt[c] = cnt.get(c, 0) + 1
        mx = max(mx, cnt[c])
    # pad lanes / Big reads share one address (broadcast): ignored
    return max(mx, 1)


def total():
    return sum(gcost(g, t) for g in range(NGRP) for t in range(DRC))


cur = total()
print("initial gather cycles", 2 * cur, "ideal", 2 * NGRP * DRC)
# variables by round/lane: swaps allowed within the same degree and round-degree class
slots_by_deg = {}
for s, j in enumerate(order):
    slots_by_deg.setdefault(cdeg[j], []).append(j)
var_checks = {j: list(Hc.indices[Hc.indptr[j]:Hc.indptr[j + 1]]) for j in range(n)}
for it in range(iters):
    T = 1.0 * (1 - it / iters) + 0.05
    mv = rnd.random()
    if mv < 0.6:  # swap two read positions of one check
        i = rnd.randrange(m)
        a, b = rnd.sample(range(DRC), 2)
        g = groups_of(i)
        old = gcost(g, a) + gcost(g, b)
        rd[i][a], rd[i][b] = rd[i][b], rd[i][a]
        d = gcost(g, a) + gcost(g, b) - old
        if not (d <= 0 or rnd.random() < np.exp(-d / T)):
            rd[i][a], rd[i][b] = rd[i][b], rd[i][a]
        else:
            cur += d
    elif mv < 0.8:  # swap two variables of equal degree (their lane slots)
        dg = rnd.choice([3, 4])
        j1, j2 = rnd.sample(slots_by_deg[dg], 2)
        aff = {groups_of(i) for i in var_checks[j1] + var_checks[j2]}
        old = sum(gcost(g, t) for g in aff for t in range(DRC))
        slot_of[j1], slot_of[j2] = slot_of[j2], slot_of[j1]
        d = sum(gcost(g, t) for g in aff for t in range(DRC)) - old
        if not (d <= 0 or rnd.random() < np.exp(-d / T)):
            slot_of[j1], slot_of[j2] = slot_of[j2], slot_of[j1]
        else:
            cur += d
    else:  # change one rotation
        rv, k = rnd.randrange(4), rnd.randrange(4)
        old_r = rot[rv][k]
        rot[rv][k] = rnd.randrange(64)
        new = total()
        d = new - cur
        if not (d <= 0 or rnd.random() < np.exp(-d / T)):
            rot[rv][k] = old_r
        else:
            cur = new
print("final gather cycles", 2 * total(), "ideal", 2 * NGRP * DRC)


# ---- phase 2: balance class degrees per group, then exact bipartite edge colouring
def hist(g):
    h = np.zeros(32, int)
    for i in range(g * 32, min(m, g * 32 + 32)):
        for j in edges[i]:
            s = slot_of[j]
            h[(s % 64 + rot[s // 64][kpos[(i, j)]]) % 32] += 1
    return h


def bal(g):
    h = hist(g)
    return int((np.maximum(h - DRC, 0) ** 2).sum())


cur = sum(bal(g) for g in range(NGRP))
print("balance cost before", cur, [int(hist(g).max()) for g in range(NGRP)])
for it in range(iters):
    T = 2.0 * (1 - it / iters) + 0.05
    if rnd.random() < 0.7:
        dg = rnd.choice([3, 4])
        j1, j2 = rnd.sample(slots_by_deg[dg], 2)
        aff = {groups_of(i) for i in var_checks[j1] + var_checks[j2]}
        old = sum(bal(g) for g in aff)
        slot_of[j1], slot_of[j2] = slot_of[j2], slot_of[j1]
        d = sum(bal(g) for g in aff) - old
        if not (d <= 0 or rnd.random() < np.exp(-d / T)):
            slot_of[j1], slot_of[j2] = slot_of[j2], slot_of[j1]
        else:
            cur += d
    else:
        rv, k = rnd.randrange(4), rnd.randrange(4)
        old_r = rot[rv][k]
        rot[rv][k] = rnd.randrange(64)
        new = sum(bal(g) for g in range(NGRP))
        d = new - cur
        if not (d <= 0 or rnd.random() < np.exp(-d / T)):
            rot[rv][k] = old_r
        else:
            cur = new
print("balance cost after", cur, [int(hist(g).max()) for g in range(NGRP)])


def colour_group(g):
    """Bipartite edge colouring (checks x classes) with max(DRC, Dmax) colours."""
    chk = list(range(g * 32, min(m, g * 32 + 32)))
    E_ = []
    for i in chk:
        for j in edges[i]:
            s = slot_of[j]
            E_.append((i, (s % 64 + rot[s // 64][kpos[(i, j)]]) % 32, j))
    C = max(DRC, int(hist(g).max()))
    at_chk = {i: {} for i in chk}     # colour -> edge idx
    at_cls = {c: {} for c in range(32)}
    col = [None] * len(E_)
    for e, (i, c, j) in enumerate(E_):
        a = next(x for x in range(C) if x not in at_chk[i])
        b = next(x for x in range(C) if x not in at_cls[c])
        if a != b:
            # flip the a/b alternating path starting at class c (a is used at c)
            path = []
            node, side, want = c, "cls", a
            while True:
                tbl = at_cls if side == "cls" else at_chk
                if want not in tbl[node]:
                    break
                f = tbl[node][want]
                path.append(f)
                fi, fc, _ = E_[f]
                node, side = (fi, "chk") if side == "cls" else (fc, "cls")
                want = b if want == a else a
            for f in path:
                fi, fc, _ = E_[f]
                del at_chk[fi][col[f]]
                del at_cls[fc][col[f]]
            for f in path:
                fi, fc, _ = E_[f]
                col[f] = b if col[f] == a else a
                at_chk[fi][col[f]] = f
                at_cls[fc][col[f]] = f
        col[e] = a
        at_chk[i][a] = e
        at_cls[c][a] = e
    return C, E_, col


tot = 0
for g in range(NGRP):
    C, E_, col = colour_group(g)
    # instructions = colours; conflicts if C > DRC: fold extra colours onto existing ones
    loads = np.zeros((DRC, 32), int)
    for e, (i, c, j) in enumerate(E_):
        loads[col[e] % DRC, c] += 1
    tot += int(loads.max(axis=1).clip(min=1).sum())
print("coloured gather cycles", 2 * tot, "ideal", 2 * NGRP * DRC)
