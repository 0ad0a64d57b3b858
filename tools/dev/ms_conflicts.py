"""Dev: LDS bank model of bp_ms_wave_kernel<double> on the C2 graph (n = 225).

Counts LDS-array cycles per shot-iteration by instruction type with the
banking rules of MI355X_MICROARCH.md §LDS, for the host layout strategy of
qdec_abi.cpp ms_layout (variables by degree, row positions annealed for the
scatter, state slots annealed for the gather) and for variants:
  --scatter-floor F   the scatter anneal's cost floor (ms_layout: 6)
  --state-writes      include the state ds_write_b128 groups in the slot anneal
Usage: python tools/dev/ms_conflicts.py [--scatter-floor 4] [--state-writes]
"""
import argparse
import os
import random
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "tests"))
from conftest import load_checks  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scatter-floor", type=int, default=6)
ap.add_argument("--state-writes", action="store_true")
ap.add_argument("--iters", type=int, default=60000)
ap.add_argument("--seed", type=int, default=1)
args = ap.parse_args()
rnd = random.Random(args.seed)

_, H = load_checks("hgp_12_3_4_s1234")
H = H.tocsr()
H.sort_indices()
m, n = H.shape
rp, ci = H.indptr, H.indices
E = rp[-1]
m_pad, n_pad = 128, 256
DRS = 10          # f64 row stride (elements)
kDC = 4
row_of = np.repeat(np.arange(m), np.diff(rp))
Hc = H.tocsc()
Hc.sort_indices()
cdeg = np.diff(Hc.indptr)
order = sorted(range(n), key=lambda j: cdeg[j])  # stable
slot_of = np.empty(n, int)
var_of_slot = -np.ones(n_pad, int)
for s, j in enumerate(order):
    slot_of[j] = s
    var_of_slot[s] = j
d3r = 0
for r in range(n_pad // 64):
    if all(var_of_slot[r * 64 + l] < 0 or cdeg[var_of_slot[r * 64 + l]] <= 3 for l in range(64)):
        d3r = r + 1
    else:
        break
D3P = d3r & ~1
cpos = np.empty(E, int)
for j in range(n):
    for k, e_row in enumerate(Hc.indices[Hc.indptr[j]:Hc.indptr[j + 1]]):
        # the CSR edge of (e_row, j)
        e = rp[e_row] + int(np.searchsorted(ci[rp[e_row]:rp[e_row + 1]], j))
        cpos[e] = k
NG = (n_pad // 64) * kDC
insts = [gi for gi in range(NG) if not (gi // kDC < D3P and gi % kDC == 3)]

# ---------------- scatter (ds_write_b64: 4 groups of 16 contiguous lanes, class = element % 16)
grp = np.array([(slot_of[ci[e]] // 64) * kDC + cpos[e] for e in range(E)])
lg = np.array([(slot_of[ci[e]] % 64) // 16 for e in range(E)])
pos = np.array([e - rp[row_of[e]] for e in range(E)])


def cls(e):
    return (row_of[e] * DRS + pos[e]) % 16


load = np.zeros((NG, 4, 16), int)
for e in range(E):
    load[grp[e], lg[e], cls(e)] += 1


def gcost(gi, floor):
    mx = load[gi].max(axis=1)
    return max(floor, int(mx.sum())) * 100000 + int((load[gi] ** 2).sum())


for it in range(40 * E):
    i = rnd.randrange(m)
    deg = rp[i + 1] - rp[i]
    e1 = rp[i] + rnd.randrange(deg)
    p2 = rnd.randrange(7)
    e2 = next((e for e in range(rp[i], rp[i + 1]) if pos[e] == p2), -1)
    if e2 == e1:
        continue
    g1, g2 = grp[e1], (grp[e2] if e2 >= 0 else -1)
    before = gcost(g1, args.scatter_floor) + (gcost(g2, args.scatter_floor) if g2 >= 0 and g2 != g1 else 0)

    def move(e, newpos):
        load[grp[e], lg[e], cls(e)] -= 1
        pos[e] = newpos
        load[grp[e], lg[e], cls(e)] += 1
    p1 = pos[e1]
    move(e1, p2)
    if e2 >= 0:
        move(e2, p1)
    after = gcost(g1, args.scatter_floor) + (gcost(g2, args.scatter_floor) if g2 >= 0 and g2 != g1 else 0)
    if after > before:
        if e2 >= 0:
            move(e2, p2)
        move(e1, p1)


def pad_groups(gi):
    pads = set()
    for l in range(64):
        j = var_of_slot[(gi // kDC) * 64 + l]
        if j < 0 or gi % kDC >= cdeg[j]:
            pads.add(l // 16)
    return pads


scatter_cycles = 0
for gi in insts:
    mx = load[gi].max(axis=1).copy()
    # pads write one dummy element in the least loaded class: + at most 1 on their groups
    pg = pad_groups(gi)
    best = min(range(16), key=lambda b: max([load[gi, h, b] for h in pg] or [0]))
    for h in pg:
        mx[h] = max(mx[h], load[gi, h, best] + 1)
    scatter_cycles += int(mx.sum())

# ---------------- row reads: 3 x b128 (conflict-free) + 1 x b64 (DRS 10: 2-way) per check round
row_cycles = 2 * (3 * 4 + 4)


# ---------------- gather (ds_read_b128: 4 groups, class = slot % 16) and state writes
def rgroup(l):
    q, h = l % 32, (l // 32) * 2
    return h + (0 if (q < 4 or 12 <= q < 16 or 20 <= q < 28) else 1)


mem, gpad = [], []
for gi in insts:
    gm = [[] for _ in range(4)]
    gp = [0] * 4
    for l in range(64):
        j = var_of_slot[(gi // kDC) * 64 + l]
        if j < 0 or gi % kDC >= cdeg[j]:
            gp[rgroup(l)] = 1
            continue
        i = Hc.indices[Hc.indptr[j] + gi % kDC]
        if i not in gm[rgroup(l)]:
            gm[rgroup(l)].append(i)
    for h in range(4):
        mem.append(gm[h])
        gpad.append(gp[h])
# state writes: check i = rc*64 + l writes slot sst[i]; ds_write_b128 groups of 8 contiguous lanes, class = slot % 8
wq = []
for rc in range(2):
    for g8 in range(8):
        wq.append([rc * 64 + g8 * 8 + t for t in range(8)])
sst = list(range(m_pad))  # checks m..m_pad-1 are pad lanes (write distinct free slots)


def qcost(q):
    cnt = [0] * 32
    mx = 0
    for i in mem[q]:
        cnt[sst[i] % 16] += 1
        mx = max(mx, cnt[sst[i] % 16])
    if gpad[q]:
        cnt[m_pad % 16] += 1
        mx = max(mx, cnt[m_pad % 16])
    return mx


def wcost(w):
    cnt = [0] * 8
    for i in wq[w]:
        cnt[sst[i] % 8] += 1
    return max(cnt)


def total():
    g = sum(qcost(q) for q in range(len(mem)))
    w = sum(wcost(x) for x in range(len(wq)))
    return g, w


app = [[] for _ in range(m_pad)]
for q in range(len(mem)):
    for i in mem[q]:
        app[i].append(q)
wapp = [i // 8 for i in range(m_pad)]
g_cur, w_cur = total()
cur = g_cur + (w_cur if args.state_writes else 0)
for it in range(args.iters):
    T = 0.6 * (1 - it / args.iters) + 0.02
    c1, c2 = rnd.randrange(m_pad), rnd.randrange(m_pad)
    if c1 == c2:
        continue
    aff = sorted(set(app[c1] + app[c2]))
    waff = sorted({wapp[c1], wapp[c2]})
    old = sum(qcost(q) for q in aff) + (sum(wcost(x) for x in waff) if args.state_writes else 0)
    sst[c1], sst[c2] = sst[c2], sst[c1]
    new = sum(qcost(q) for q in aff) + (sum(wcost(x) for x in waff) if args.state_writes else 0)
    d = new - old
    if d <= 0 or rnd.random() < np.exp(-d / T):
        cur += d
    else:
        sst[c1], sst[c2] = sst[c2], sst[c1]
g_cyc, w_cyc = total()
g_cyc *= 1
print(f"D3P={D3P} instructions={len(insts)}")
print(f"scatter  array cycles {scatter_cycles:4d}  (ideal {4 * len(insts)})  floor {args.scatter_floor}")
print(f"gather   array cycles {g_cyc:4d}  (ideal {4 * len(insts)})")
print(f"state wr array cycles {w_cyc:4d}  (ideal 16)")
print(f"row rd   array cycles {row_cycles:4d}  (ideal 24 + 4)")
tot = scatter_cycles + g_cyc + w_cyc + row_cycles
ideal = 8 * len(insts) + 16 + 28
print(f"total {tot}  ideal {ideal}  conflicts {tot - ideal}")
