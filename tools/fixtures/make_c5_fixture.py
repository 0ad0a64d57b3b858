"""Build BASELINE config 5 as named -- the PSL(2,16) Cayley-graph lifted-product
code lifted_product_code_pgl2(1, 4, 2, double_cover=False, seed=1) (reference
python/qldpc/lifted_product_code.py:411-453, Morgenstern generators :164-203) --
with this package's own construction (exp_ldpc_amd/lifted.py), and store its
checks and logicals as test fixtures:

  tests/golden/lp_pgl2_1_4_2_s1_checks.npz     Hx, Hz (24,480 x 53,040 each)
  tests/golden/lp_pgl2_1_4_2_s1_logicals.npz   Lx, Lz (4,080 x 53,040, CSR)

double_cover=False is required: with the default the reference's wrapper sizes
the local codes for the single-vertex base graph but builds the double cover,
and raises its own block-length error (lifted_product_code.py:426 vs :288).
The logicals come from the threaded GF(2) elimination (gf2.css_logicals, a few
minutes); the reference would use galois, which is absent here, so the fixture
is pinned by the CSS relations checked below, not by reference output.

Usage: python tools/fixtures/make_c5_fixture.py
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")
NAME = "lp_pgl2_1_4_2_s1"


def _save_pair(path, a_name, A, b_name, B):
    A, B = sp.csr_matrix(A), sp.csr_matrix(B)
    np.savez_compressed(path, **{f"{a_name}_indptr": A.indptr.astype(np.int32), f"{a_name}_indices": A.indices.astype(np.int32),
                                 f"{a_name}_shape": np.array(A.shape), f"{b_name}_indptr": B.indptr.astype(np.int32),
                                 f"{b_name}_indices": B.indices.astype(np.int32), f"{b_name}_shape": np.array(B.shape)})


def main():
    from exp_ldpc_amd import gf2
    from exp_ldpc_amd.lifted import lifted_product_code_pgl2
    code = lifted_product_code_pgl2(1, 4, 2, compute_logicals=False, seed=1, double_cover=False)
    hx, hz = sp.csr_matrix(code.checks.x), sp.csr_matrix(code.checks.z)
    print("checks", hx.shape, hz.shape, hx.nnz, hz.nnz, flush=True)
    _save_pair(os.path.join(GOLDEN, f"{NAME}_checks.npz"), "hx", hx, "hz", hz)
    t = time.time()
    lx, lz = gf2.css_logicals(hx, hz)
    lx, lz = sp.csr_matrix(lx), sp.csr_matrix(lz)
    print(f"logicals k={lz.shape[0]} in {time.time() - t:.0f}s, nnz Lz {lz.nnz}, Lx {lx.nnz}", flush=True)
    assert not ((hx @ lz.T).toarray() % 2).any() and not ((hz @ lx.T).toarray() % 2).any()
    pair = (lx @ lz.T).toarray() % 2
    assert np.array_equal(pair, np.eye(lz.shape[0], dtype=pair.dtype))
    _save_pair(os.path.join(GOLDEN, f"{NAME}_logicals.npz"), "lx", lx, "lz", lz)


if __name__ == "__main__":
    main()
