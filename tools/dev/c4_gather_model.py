"""Dev: state-gather bank model of bp_ms_lds_kernel (C4, hgp_80_3_4_s2025).

The variable pass reads one float4 state per edge at row r's half h = bit 3 of
r: ds_read_b128, 4 groups of 16 lanes ({0-3,12-15,20-27}, {4-11,16-19,28-31},
+32), class = (2 r + h) mod 16; distinct rows of one class in one group
conflict.  Reports LDS-array cycles per iteration of all gathers for the
identity check -> row map and after an anneal of a row permutation.
Usage: python tools/dev/c4_gather_model.py [iters]
"""
import math
import os
import random
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "tests"))
from conftest import load_checks  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 300000
rnd = random.Random(7)
_, H = load_checks("hgp_80_3_4_s2025")
Hc = H.tocsc()
Hc.sort_indices()
m, n = H.shape
NT, DC = 1024, 4
rounds = (n + NT - 1) // NT


def rgroup(l):
    q, h = l % 32, (l // 32) * 2
    return h + (0 if (q < 4 or 12 <= q < 16 or 20 <= q < 28) else 1)


# instructions: (round, wave, k) -> per group list of checks (or pad dummy rows)
inst = []
for r in range(rounds):
    for w in range(NT // 64):
        for k in range(DC):
            groups = [[] for _ in range(4)]
            for l in range(64):
                j = r * NT + w * 64 + l
                if j < n and k < Hc.indptr[j + 1] - Hc.indptr[j]:
                    groups[rgroup(l)].append(("c", int(Hc.indices[Hc.indptr[j] + k])))
                else:
                    groups[rgroup(l)].append(("d", m + l // 8))  # dummy rows past m
            inst.append(groups)
row_of = list(range(m))


def cls(row):
    return (2 * row + ((row >> 3) & 1)) % 16


def gcost(q, g):
    seen = set()
    cnt = [0] * 16
    for kind, x in inst[q][g]:
        row = row_of[x] if kind == "c" else x
        if row in seen:
            continue
        seen.add(row)
        cnt[cls(row)] += 1
    return max(max(cnt), 1) * 1000 + sum(c * c for c in cnt)


cost = {(q, g): gcost(q, g) for q in range(len(inst)) for g in range(4)}
print("instructions", len(inst), "gather cycles", sum(v // 1000 for v in cost.values()), "ideal", 4 * len(inst))
app = [set() for _ in range(m)]
for q in range(len(inst)):
    for g in range(4):
        for kind, x in inst[q][g]:
            if kind == "c":
                app[x].add((q, g))
cur = sum(cost.values())
for it in range(iters):
    T = 30.0 * (1 - it / iters) + 1.0
    a, b = rnd.randrange(m), rnd.randrange(m)
    if a == b or cls(row_of[a]) == cls(row_of[b]):
        continue
    aff = app[a] | app[b]
    old = sum(cost[x] for x in aff)
    row_of[a], row_of[b] = row_of[b], row_of[a]
    new = {x: gcost(*x) for x in aff}
    d = sum(new.values()) - old
    if d <= 0 or rnd.random() < math.exp(-d / T):
        cost.update(new)
        cur += d
    else:
        row_of[a], row_of[b] = row_of[b], row_of[a]
    if it % 100000 == 0:
        print(it, sum(v // 1000 for v in cost.values()), flush=True)
print("annealed gather cycles", sum(v // 1000 for v in cost.values()), "ideal", 4 * len(inst))
