"""Logical operators of BASELINE config 4's code as a test/bench fixture:
biregular_hgp(80, 3, 4, seed=2025) (n = 10^4; its checks are the
reference-generated tests/golden/hgp_80_3_4_s2025_checks.npz), logicals from
this package's threaded GF(2) elimination (gf2.css_logicals; the reference's
get_logicals uses galois, absent here), pinned by the CSS relations below.

  tests/golden/hgp_80_3_4_s2025_logicals.npz   Lx, Lz (CSR)

Usage: python tools/fixtures/make_c4_logicals.py
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
GOLDEN = os.path.join(REPO, "tests", "golden")
NAME = "hgp_80_3_4_s2025"


def main():
    from conftest import load_checks
    from exp_ldpc_amd import gf2
    hx, hz = load_checks(NAME)
    lx, lz = gf2.css_logicals(hx, hz)
    lx, lz = sp.csr_matrix(lx), sp.csr_matrix(lz)
    assert not ((hx @ lz.T).toarray() % 2).any() and not ((hz @ lx.T).toarray() % 2).any()
    assert lx.shape[0] == lz.shape[0] and not np.all(((lx @ lz.T).toarray() % 2) == 0)
    np.savez_compressed(os.path.join(GOLDEN, f"{NAME}_logicals.npz"),
                        lx_indptr=lx.indptr.astype(np.int32), lx_indices=lx.indices.astype(np.int32),
                        lx_shape=np.array(lx.shape), lz_indptr=lz.indptr.astype(np.int32),
                        lz_indices=lz.indices.astype(np.int32), lz_shape=np.array(lz.shape))
    print(f"k = {lz.shape[0]}, nnz Lz {lz.nnz}, Lx {lx.nnz}")


if __name__ == "__main__":
    main()
