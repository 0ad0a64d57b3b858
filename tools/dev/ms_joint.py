"""Dev: joint LDS-layout anneal model for bp_ms_wave_kernel<double> (C2 graph).

State: variable lane slots (swaps inside a degree class), v2c row positions
(0..DRC-1 per check), state slots (permutation of m_pad).  Cost = LDS-array
cycles per shot-iteration of the v2c scatter (ds_write_b64), the state gather
(ds_read_b128), the state writes (ds_write_b128) and the row reads
(constant), by the banking rules of MI355X_MICROARCH.md §LDS.
Usage: python tools/dev/ms_joint.py [iters] [seed]
"""
import math
import os
import random
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "tests"))
from conftest import load_checks  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
rnd = random.Random(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
_, H = load_checks("hgp_12_3_4_s1234")
H = H.tocsr()
H.sort_indices()
m, n = H.shape
rp, ci = H.indptr, H.indices
E = int(rp[-1])
Hc = H.tocsc()
Hc.sort_indices()
cdeg = np.diff(Hc.indptr)
m_pad, n_pad, DRS, kDC = 128, 256, 10, 4
DRC = int(np.diff(rp).max())
row_of = np.repeat(np.arange(m), np.diff(rp))
order = sorted(range(n), key=lambda j: cdeg[j])
slot_of = [0] * n
var_of_slot = [-1] * n_pad
for s, j in enumerate(order):
    slot_of[j] = s
    var_of_slot[s] = j
D3P = 2
cpos = [0] * E
edge_of = {}
for i in range(m):
    for e in range(rp[i], rp[i + 1]):
        edge_of[(i, int(ci[e]))] = e
col_edges = [[] for _ in range(n)]
for j in range(n):
    for k, i in enumerate(Hc.indices[Hc.indptr[j]:Hc.indptr[j + 1]]):
        e = edge_of[(int(i), j)]
        cpos[e] = k
        col_edges[j].append(e)
pos = [e - rp[row_of[e]] for e in range(E)]
sst = list(range(m_pad))
NG = 16
insts = [gi for gi in range(NG) if not (gi // kDC < D3P and gi % kDC == 3)]


def rgroup(l):
    q, h = l % 32, (l // 32) * 2
    return h + (0 if (q < 4 or 12 <= q < 16 or 20 <= q < 28) else 1)


def inst_cost(gi):
    """scatter + gather array cycles of instruction (rv, k) = gi."""
    rv, k = divmod(gi, kDC)
    sc = [[0] * 16 for _ in range(4)]
    gm = [set() for _ in range(4)]
    padw = [False] * 4
    padr = [False] * 4
    for l in range(64):
        j = var_of_slot[rv * 64 + l]
        if j < 0 or k >= cdeg[j]:
            padw[l // 16] = True
            padr[rgroup(l)] = True
            continue
        e = col_edges[j][k]
        i = row_of[e]
        sc[l // 16][(i * DRS + pos[e]) % 16] += 1
        gm[rgroup(l)].add(i)
    # pads: one dummy element, least loaded class over the pad groups
    best = min(range(16), key=lambda b: max([sc[h][b] for h in range(4) if padw[h]] or [0]))
    s_cyc = 0
    for h in range(4):
        mx = max(sc[h])
        if padw[h]:
            mx = max(mx, sc[h][best] + 1)
        s_cyc += max(mx, 1)
    g_cyc = 0
    for h in range(4):
        cnt = [0] * 16
        for i in gm[h]:
            cnt[sst[i] % 16] += 1
        if padr[h]:
            cnt[m_pad % 16] += 1
        g_cyc += max(max(cnt), 1)
    return s_cyc, g_cyc


def wcost(w):
    cnt = [0] * 8
    for t in range(8):
        cnt[sst[w * 8 + t] % 8] += 1
    return max(cnt)


ic = {gi: inst_cost(gi) for gi in insts}
wc = [wcost(w) for w in range(16)]


def total():
    s = sum(v[0] for v in ic.values())
    g = sum(v[1] for v in ic.values())
    return s, g, sum(wc)


def show(tag):
    s, g, w = total()
    print(f"{tag}: scatter {s} gather {g} state-wr {w} rows 32 -> total {s + g + w + 32}")


show("initial")
inst_of_edge = [(slot_of[int(ci[e])] // 64) * kDC + cpos[e] for e in range(E)]
checks_insts = [sorted({inst_of_edge[e] for e in range(rp[i], rp[i + 1])}) for i in range(m)]
same_deg = {}
for j in range(n):
    same_deg.setdefault(int(cdeg[j]), []).append(j)
cur = sum(sum(v) for v in ic.values()) + sum(wc)
for it in range(iters):
    T = 0.4 * (1 - it / iters) + 0.01
    mv = rnd.random()
    if mv < 0.45:    # row position swap
        i = rnd.randrange(m)
        e1 = rp[i] + rnd.randrange(rp[i + 1] - rp[i])
        p2 = rnd.randrange(DRC)
        e2 = next((e for e in range(rp[i], rp[i + 1]) if pos[e] == p2), -1)
        if e2 == e1:
            continue
        aff = {(slot_of[int(ci[e1])] // 64) * kDC + cpos[e1]}
        if e2 >= 0:
            aff.add((slot_of[int(ci[e2])] // 64) * kDC + cpos[e2])
        undo = lambda: None
        p1 = pos[e1]
        pos[e1] = p2
        if e2 >= 0:
            pos[e2] = p1

        def undo():
            pos[e1] = p1
            if e2 >= 0:
                pos[e2] = p2
        wa = []
    elif mv < 0.75:  # variable swap (same degree)
        dg = rnd.choice(list(same_deg))
        if len(same_deg[dg]) < 2:
            continue
        j1, j2 = rnd.sample(same_deg[dg], 2)
        aff = {(slot_of[j] // 64) * kDC + k for j in (j1, j2) for k in range(dg)}
        s1, s2 = slot_of[j1], slot_of[j2]
        slot_of[j1], slot_of[j2] = s2, s1
        var_of_slot[s1], var_of_slot[s2] = j2, j1
        aff |= {(slot_of[j] // 64) * kDC + k for j in (j1, j2) for k in range(dg)}

        def undo():
            slot_of[j1], slot_of[j2] = s1, s2
            var_of_slot[s1], var_of_slot[s2] = j1, j2
        wa = []
    else:            # state slot swap
        c1, c2 = rnd.randrange(m_pad), rnd.randrange(m_pad)
        if c1 == c2:
            continue
        aff = set()
        for c in (c1, c2):
            if c < m:
                for e in range(rp[c], rp[c + 1]):
                    aff.add((slot_of[int(ci[e])] // 64) * kDC + cpos[e])
        sst[c1], sst[c2] = sst[c2], sst[c1]

        def undo():
            sst[c1], sst[c2] = sst[c2], sst[c1]
        wa = sorted({c1 // 8, c2 // 8})
    aff = [a for a in aff if a in ic]
    old = sum(sum(ic[a]) for a in aff) + sum(wc[w] for w in wa)
    new_ic = {a: inst_cost(a) for a in aff}
    new_wc = {w: wcost(w) for w in wa}
    d = sum(sum(v) for v in new_ic.values()) + sum(new_wc.values()) - old
    if d <= 0 or rnd.random() < math.exp(-d / T):
        ic.update(new_ic)
        for w, v in new_wc.items():
            wc[w] = v
        cur += d
    else:
        undo()
    if it % 50000 == 0:
        show(f"it {it}")
show("final")
