"""Dev: LDS-array cycle model of bp_ms_lds64_kernel's per-edge state accesses on
the C4 graph for the library's check-state slots (qd_graph_lds64_slots_copy),
with the banking measured by tools/dev/lds_atomic_probe.hip on gfx950:
  ds_read_b64 (m1, m2)       2 x 32-lane groups, key slot mod 32, 2 cycles base
  ds_min(_rtn)_u64 (m1, m2)  4 x 16-lane groups, key slot mod 16, 4 cycles base
  ds_read_b32 / ds_xor_b32   2 x 32-lane groups, key (slot >> 5) mod 32, 2 cycles base
A group costs the most distinct addresses on one bank (atomics: lanes).  Prints
the model's cycles per iteration and its conflict share, for the natural order
and the library's slots."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import load_checks  # noqa: E402

from exp_ldpc_amd import _abi  # noqa: E402

hx, hz = load_checks("hgp_80_3_4_s2025")
H = hz.tocsr()
H.sort_indices()
m, n = H.shape
lib = _abi.load()
rp = np.ascontiguousarray(H.indptr, np.int32)
ci = np.ascontiguousarray(H.indices, np.int32)
h = C.c_void_p()
_abi.check(lib.qd_graph_create_host(m, n, _abi.ptr(rp), _abi.ptr(ci), n, 1, C.byref(h)), "create")
et = np.zeros(4 * n, np.uint16)
chk = np.zeros(m, np.uint16)
_abi.check(lib.qd_graph_lds64_slots_copy(h, _abi.ptr(et), _abi.ptr(chk)), "slots")
lib.qd_graph_destroy(h)
slot_of = np.empty(m, np.int64)
slot_of[chk] = np.arange(m)
Hc = H.tocsc()
Hc.sort_indices()
colchk = np.full((4, n), -1)
for j in range(n):
    rows = Hc.indices[Hc.indptr[j]:Hc.indptr[j + 1]]
    colchk[:rows.size, j] = rows
# lanes' checks per instruction (wave, round, edge): list of 64 entries (-1 = inactive)
insts = []
for w in range(16):
    for r in range((n + 1023) // 1024):
        for k in range(4):
            js = [r * 1024 + ((64 * w + l) * 67) % 1024 for l in range(64)]
            cs = np.array([colchk[k, j] if j < n else -1 for j in js])
            if (cs >= 0).any():
                insts.append(cs)


def group_cost(s, key_mod, shift, distinct):
    s = s[s >= 0]
    if s.size == 0:
        return 0
    if distinct:
        s = np.unique(s)
    return np.bincount((s >> shift) % key_mod, minlength=key_mod).max()


def model(slot):
    tot = base = 0.0
    for cs in insts:
        s = np.where(cs >= 0, slot[np.maximum(cs, 0)], -1)
        for g in range(2):  # reads: 2 x 32, key mod 32, distinct addresses; x2 (m1, m2)
            c = group_cost(s[32 * g:32 * g + 32], 32, 0, True)
            tot += 2 * c
            base += 2 * (c > 0)
        for g in range(4):  # u64 atomics: 4 x 16, key mod 16; x2 (m1, m2)
            c = group_cost(s[16 * g:16 * g + 16], 16, 0, False)
            tot += 2 * c
            base += 2 * (c > 0)
        for g in range(2):  # parw read (+ xors when taken): words, key mod 32
            c = group_cost(s[32 * g:32 * g + 32], 32, 5, True)
            tot += c
            base += (c > 0)
    return tot, 1 - base / tot


for name, sl in (("natural", np.arange(m)), ("library", slot_of)):
    t, cf = model(sl)
    print(f"{name:8s} model cycles/iteration-CU {t:9.0f}  conflict share {cf:.3f}")

# inherent part: lanes of one atomic group on the same check (same address)
dup = tot = 0
for cs in insts:
    for g in range(4):
        s = cs[16 * g:16 * g + 16]
        s = s[s >= 0]
        tot += s.size
        dup += s.size - np.unique(s).size
print(f"atomic lanes {tot}, lanes whose check already appears in their 16-lane group: {dup}")
