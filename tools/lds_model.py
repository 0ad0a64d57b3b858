"""LDS cycle model of the BP wave kernel's per-iteration LDS traffic
(MI355X_MICROARCH.md § LDS bank rules), for layout experiments on the host.

cost(instr, addrs): addrs = per-lane byte addresses (None = lane inactive).
"""
import sys
import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])

B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128_GROUPS += [[l + 32 for l in g] for g in B128_GROUPS]


def _groups(kind):
    if kind in ("r32", "r64", "w32"):
        return [list(range(0, 32)), list(range(32, 64))]
    if kind == "r128":
        return B128_GROUPS
    if kind in ("w64",):
        return [list(range(16 * q, 16 * q + 16)) for q in range(4)]
    if kind in ("w128", "w96"):
        return [list(range(8 * q, 8 * q + 8)) for q in range(8)]
    raise ValueError(kind)


def cost(kind, addrs):
    width = {"r32": 1, "w32": 1, "r64": 2, "w64": 2, "r128": 4, "w128": 4, "w96": 3}[kind]
    nbanks = 64 if kind in ("r64", "r128") else 32
    total = 0
    for g in _groups(kind):
        banks = {}
        for l in g:
            a = addrs[l]
            if a is None:
                continue
            for d in range(width):
                dw = a // 4 + d
                banks.setdefault(dw % nbanks, set()).add(dw)
        total += max((len(s) for s in banks.values()), default=1)
    floor = {"w32": 4, "w64": 6, "w128": 13, "w96": 10}.get(kind, 0)
    return max(total, floor)


def current_design(H, DRS=12, DCS=4, RC=2, RV=4, DRC=7):
    """Cycles per iteration of the current kernel (scatter c2v, scatter v2c,
    byte syndrome gathers), LDS only."""
    H = H.tocsr()
    m, n = H.shape
    m_pad, n_pad = RC * 64, RV * 64
    rows = [list(H.indices[H.indptr[i]:H.indptr[i + 1]]) for i in range(m)]
    cols = [[] for _ in range(n)]
    for i, r in enumerate(rows):
        for j in r:
            cols[j].append(i)
    v2c0 = 0
    c2v0 = (m_pad * DRS + 64) * 4
    xh0 = c2v0 + (n_pad * DCS + 64) * 4
    cyc = {}
    # check pass: read row (DRC <= 8 -> 2 b128), scatter c2v
    for rc in range(RC):
        for h in range(2):
            cyc["chk_read"] = cyc.get("chk_read", 0) + cost("r128", [v2c0 + ((rc * 64 + l) * DRS + 4 * h) * 4 for l in range(64)])
        for k in range(DRC):
            ad = []
            for l in range(64):
                i = rc * 64 + l
                if i < m and k < len(rows[i]):
                    j = rows[i][k]
                    ad.append(c2v0 + (j * DCS + cols[j].index(i)) * 4)
                else:
                    ad.append(c2v0 + (n_pad * DCS + l) * 4)
            cyc["chk_scatter"] = cyc.get("chk_scatter", 0) + cost("w32", ad)
    for rv in range(RV):
        cyc["var_read"] = cyc.get("var_read", 0) + cost("r128", [c2v0 + ((rv * 64 + l) * DCS) * 4 for l in range(64)])
        for k in range(4):
            ad = []
            for l in range(64):
                j = rv * 64 + l
                if j < n and k < len(cols[j]):
                    i = cols[j][k]
                    ad.append(v2c0 + (i * DRS + rows[i].index(j)) * 4)
                else:
                    ad.append(v2c0 + (m_pad * DRS + l) * 4)
            cyc["var_scatter"] = cyc.get("var_scatter", 0) + cost("w32", ad)
        cyc["xh_write"] = cyc.get("xh_write", 0) + 4  # ds_write_b8, contiguous
    for rc in range(RC):
        for k in range(DRC):
            ad = []
            for l in range(64):
                i = rc * 64 + l
                j = rows[i][k] if (i < m and k < len(rows[i])) else n_pad + l
                ad.append(xh0 + (j // 4) * 4)  # byte reads: bank of the dword
            cyc["syn_gather"] = cyc.get("syn_gather", 0) + cost("r32", ad)
    cyc["total"] = sum(cyc.values())
    return cyc


if __name__ == "__main__":
    d = np.load(sys.argv[1] if len(sys.argv) > 1 else
                __file__.rsplit("/tools/", 1)[0] + "/tests/golden/hgp_12_3_4_s1234_checks.npz")
    import scipy.sparse as sp
    H = sp.csr_matrix((np.ones(len(d["hz_indices"])), d["hz_indices"], d["hz_indptr"]), shape=tuple(d["hz_shape"]))
    print(current_design(H))


def compressed_design(H, DRS=12, RC=2, RV=4, perm_r=None, perm_c=None, state_stride=2):
    """Compressed min-sum: check lanes read their v2c row and write a 2-dword
    state; variable lanes gather the states of their checks and scatter v2c.
    perm_r[i] / perm_c[j]: lane slot of check i / variable j."""
    H = H.tocsr()
    m, n = H.shape
    m_pad, n_pad = RC * 64, RV * 64
    pr = np.arange(m) if perm_r is None else np.asarray(perm_r)
    pc = np.arange(n) if perm_c is None else np.asarray(perm_c)
    rows = [list(H.indices[H.indptr[i]:H.indptr[i + 1]]) for i in range(m)]
    cols = [[] for _ in range(n)]
    for i, r in enumerate(rows):
        for j in r:
            cols[j].append(i)
    inv_c = {int(pc[j]): j for j in range(n)}
    v2c0 = 0
    st0 = (m_pad * DRS + 64) * 4
    cyc = {"chk_read": 4 * RC * 2 * 0}
    for rc in range(RC):
        for h in range(2):
            cyc["chk_read"] += cost("r128", [v2c0 + ((rc * 64 + l) * DRS + 4 * h) * 4 for l in range(64)])
        cyc["state_write"] = cyc.get("state_write", 0) + cost("w64", [st0 + (rc * 64 + l) * state_stride * 4 for l in range(64)])
    for rv in range(RV):
        for k in range(4):
            ad_g, ad_s = [], []
            for l in range(64):
                j = inv_c.get(rv * 64 + l)
                if j is not None and k < len(cols[j]):
                    i = cols[j][k]
                    ad_g.append(st0 + int(pr[i]) * state_stride * 4)
                    ad_s.append(v2c0 + (int(pr[i]) * DRS + rows[i].index(j)) * 4)
                else:
                    ad_g.append(ad_g[0] if ad_g else st0)
                    ad_s.append(v2c0 + (m_pad * DRS + l) * 4)
            cyc["state_gather"] = cyc.get("state_gather", 0) + cost("r64", ad_g)
            cyc["var_scatter"] = cyc.get("var_scatter", 0) + cost("w32", ad_s)
    cyc["total"] = sum(cyc.values())
    return cyc
