"""HGP code sources (exp_ldpc_amd/hgp.py) against fixtures the reference itself
generated (tests/golden/make_golden.py), plus the reference's own property tests
(tests/test_random_biregular_graph.py:6-61, tests/test_hypergraph_product_code.py).
CPU only."""
import os

import numpy as np
import pytest
import scipy.sparse as sp

from exp_ldpc_amd import gf2
from exp_ldpc_amd.hgp import biregular_hgp, homological_product, random_biregular_graph, remove_short_cycles, search_cycle

GOLD = os.path.join(os.path.dirname(__file__), "golden")
GRAPH_SEEDS = [0x59824c5a, 0x9dca707a, 0xe0218aa8, 0x81da8035]
GRAPH_SHAPES = [(27, 3, 4), (10, 5, 6), (21, 7, 8), (27, 9, 10)]


def _edges(g):
    return np.array(sorted((min(u, v), max(u, v)) for u, v in g.edges()), dtype=np.int64)


def _same_csr(m, f, key):
    m = sp.csr_matrix(m)
    return (np.array_equal(m.indptr, f[f"{key}_indptr"]) and np.array_equal(m.indices, f[f"{key}_indices"])
            and tuple(m.shape) == tuple(f[f"{key}_shape"]))


@pytest.mark.parametrize("name,kw", [
    ("hgp_12_3_4_s1234", dict(num_data=12, data_degree=3, check_degree=4, seed=1234)),
    ("hgp_12_3_4_s7", dict(num_data=12, data_degree=3, check_degree=4, seed=7)),
    ("hgp_24_3_4_s11", dict(num_data=24, data_degree=3, check_degree=4, seed=11)),
    ("hgp_36_3_4_s42_g4", dict(num_data=36, data_degree=3, check_degree=4, seed=42, girth_bound=4)),
    ("hgp_80_3_4_s2025", dict(num_data=80, data_degree=3, check_degree=4, seed=2025)),
])
def test_biregular_hgp_matches_reference(name, kw):
    code = biregular_hgp(**kw)
    f = np.load(os.path.join(GOLD, f"{name}_checks.npz"))
    assert _same_csr(code.checks.x, f, "hx") and _same_csr(code.checks.z, f, "hz")


@pytest.mark.parametrize("shape", GRAPH_SHAPES)
@pytest.mark.parametrize("seed", GRAPH_SEEDS)
def test_random_biregular_graph_matches_reference(shape, seed):
    lv, rdeg, ldeg = shape
    g = random_biregular_graph(lv, lv * ldeg // rdeg, rdeg, ldeg, seed=seed)
    ref = np.load(os.path.join(GOLD, "graphs.npz"))[f"rbg_{lv}_{rdeg}_{ldeg}_{seed}"]
    assert np.array_equal(_edges(g), ref)
    for v, d in g.degree():  # biregular, reference test :6-14
        assert d == (rdeg if g.nodes[v]["bipartite"] == 0 else ldeg)


@pytest.mark.parametrize("seed", GRAPH_SEEDS[:2])
def test_remove_short_cycles_matches_reference(seed):
    g = random_biregular_graph(102, 136, 3, 4, seed=seed)
    remove_short_cycles(g, 4, seed=seed - 42, patience=10000)
    ref = np.load(os.path.join(GOLD, "graphs.npz"))[f"girth4_102_3_4_{seed}"]
    assert np.array_equal(_edges(g), ref)
    for v in g.nodes:  # girth > 4 (reference :16-19)
        assert search_cycle(g, v, 2) is None


def test_search_cycle_on_hexagon():
    import networkx as nx
    g = nx.cycle_graph(6)
    assert search_cycle(g, 0, 2) is None
    length, edge = search_cycle(g, 0, 3)
    assert length == 6 and edge is not None


def test_homological_product_commutes_and_counts():
    code = biregular_hgp(12, 3, 4, seed=1234, compute_logicals=True, check_complex=True)
    hx, hz = code.checks.x.toarray(), code.checks.z.toarray()
    assert not np.any((hx @ hz.T) % 2)
    assert code.num_logicals == 9  # README.md:49-50, SURVEY §6 probe
    lx, lz = code.logicals.x.astype(np.int64), code.logicals.z.astype(np.int64)
    assert not np.any((hz @ lx.T) % 2) and not np.any((hx @ lz.T) % 2)
    assert np.array_equal((lz @ lx.T) % 2, np.eye(9, dtype=np.int64))


def test_homological_product_shapes():
    rng = np.random.default_rng(3)
    A = sp.csr_matrix(rng.integers(0, 2, size=(5, 7)))
    B = sp.csr_matrix(rng.integers(0, 2, size=(4, 6)))
    code = homological_product(A, B, check_complex=True, compute_logicals=True)
    assert code.num_qubits == 5 * 6 + 7 * 4
    assert code.checks.x.shape[0] == 7 * 6 and code.checks.z.shape[0] == 5 * 4
    rx, rz = gf2.rank(code.checks.x.toarray()), gf2.rank(code.checks.z.toarray())
    assert code.num_logicals == code.num_qubits - rx - rz
