"""Hypergraph-product code sources (host side, offline): the random
(dv, dc)-biregular Tanner graph, short-cycle surgery, the homological product
and the ``biregular_hgp`` generator the north-star config is built from
(``scripts/generate_hgp_code.py 4 3 12`` -> ``biregular_hgp(12, 3, 4)``).

Reference behaviour restated here (the random draws go through the same
networkx / numpy / scipy calls in the same order, so a given seed yields the
same code as the reference; pinned by ``tests/golden/hgp_*``):

* ``random_biregular_graph``  -- ``python/qldpc/random_biregular_graph.py:14-89``
  (configuration model, then random endpoint swaps until no multi-edge is left)
* ``remove_short_cycles``     -- ``random_biregular_graph.py:121-178``
  (Alon-Rodeh BFS cycle search ``:91-118``, degree-weighted edge swaps)
* ``homological_product``     -- ``python/qldpc/homological_product_code.py:64-103``
* ``biregular_hgp`` / ``random_test_hgp`` -- ``python/qldpc/hypergraph_product_code.py:7-40``

Logicals are computed with this package's own GF(2) elimination
(``gf2.css_logicals``) instead of galois; they span the same spaces as the
reference's (``homological_product_code.py:37-60``) but the basis may differ.
Nothing here runs on the GPU.
"""
from __future__ import annotations

import warnings
from collections import deque

import numpy as np
import scipy.sparse as sp

from .codes import QuantumCode, QuantumCodeChecks, QuantumCodeLogicals

__all__ = ["random_biregular_graph", "remove_short_cycles", "search_cycle", "homological_product",
           "code_from_boundary_maps", "biregular_hgp", "random_test_hgp"]


def _nx():
    import networkx as nx
    return nx


def _sorted_pair(a, b):
    return (a, b) if a < b else (b, a)


def _data_check_pair(graph, e):
    """Orient an edge as (data node, check node) (reference :11-12)."""
    u, v = e[0], e[1]
    return (u, v) if graph.nodes[v]["bipartite"] == 1 else (v, u)


def _multi_edge_surplus(graph, data_nodes):
    """One (data, check) entry per surplus parallel edge, scanned data node by
    data node in adjacency order (reference :45-52)."""
    surplus = []
    for d in data_nodes:
        for c in graph.neighbors(d):
            k = graph.number_of_edges(d, c)
            surplus.extend([(d, c)] * (k - 1))
    return surplus


def random_biregular_graph(num_checks: int, num_data: int, data_degree: int, check_degree: int, seed=None,
                           graph_multiedge_retries=None):
    """Random bipartite graph, every data node of degree ``data_degree`` and every
    check node of degree ``check_degree``; data nodes are ``bipartite=0``.

    Configuration model first; surplus parallel edges are then swapped against
    uniformly chosen edges (a <-> b endpoint exchange keeps all degrees) for up to
    ``graph_multiedge_retries`` rounds (reference :14-89)."""
    nx = _nx()
    retries = 100 if graph_multiedge_retries is None else graph_multiedge_retries
    if num_checks * check_degree != num_data * data_degree:
        raise RuntimeError("Number of data bits incompatible with data and check degrees")
    g = nx.bipartite.configuration_model([data_degree] * num_data, [check_degree] * num_checks, seed=seed,
                                         create_using=nx.MultiGraph())
    rng = np.random.default_rng(seed=seed)
    data_nodes = [v for v, attrs in g.nodes(data=True) if attrs["bipartite"] == 0]
    for _ in range(retries):
        surplus = _multi_edge_surplus(g, data_nodes)
        if not surplus:
            break
        partners = rng.choice(list(g.edges()), size=len(surplus), replace=False)
        drop, add = [], []
        for a, b in zip(surplus, partners):
            b_key = _sorted_pair(b[0], b[1])
            if b_key in drop:  # partner already consumed by an earlier swap this round
                continue
            drop += [_sorted_pair(a[0], a[1]), b_key]
            add += [_sorted_pair(a[0], b[1]), _sorted_pair(b[0], a[1])]
        for e in drop:
            g.remove_edge(*e, key=None)
        g.add_edges_from(add)
    else:
        raise RuntimeError("Unable to remove multiedges from the graph")
    return nx.Graph(g)


def search_cycle(graph, source, depth_limit: int):
    """BFS from ``source`` to ``depth_limit`` levels; on the first non-tree edge
    (u, w) with level(u) <= level(w) return ``(2*(level(u)+1), (u, w))``, else None
    (Alon-Rodeh; reference ``_search_cycle`` :91-118)."""
    level = {source: 0}
    todo = deque([source])
    while todo:
        u = todo.popleft()
        lu = level[u]
        for w in graph.neighbors(u):
            lw = level.get(w)
            if lw is None:
                level[w] = lu + 1
                if lu + 1 < depth_limit:
                    todo.append(w)
            elif lu <= lw:
                return (2 * (lu + 1), (u, w))
    return None


def remove_short_cycles(graph, girth_bound: int, seed=None, patience=1000000) -> None:
    """Swap edges in place until the girth exceeds ``girth_bound``
    (reference :121-178): pick a random data node, find a short cycle through it,
    and exchange one of its edges with an edge sampled uniformly (vertex weighted
    by degree, then one of its edges) when that creates no multi-edge."""
    nx = _nx()
    from scipy.stats import rv_discrete
    depth = girth_bound // 2
    data_view = nx.subgraph_view(graph, filter_node=lambda v: graph.nodes[v]["bipartite"] == 0)
    data_nodes = np.array(data_view.nodes())
    rng = np.random.default_rng(seed=seed)
    check_every = data_nodes.shape[0] * 10
    verts = np.fromiter(graph.nodes(), dtype=np.int32)
    deg = np.fromiter((graph.degree(v) for v in verts), dtype=np.int32)
    pick_vertex = rv_discrete(values=(verts, deg / np.sum(deg)))

    def girth_ok():
        return all(search_cycle(graph, v, depth_limit=depth) is None for v in data_nodes)

    for t in range(patience):
        if t % check_every == 0 and girth_ok():
            return
        hit = search_cycle(graph, rng.choice(data_nodes), depth_limit=depth)
        if hit is None:
            continue
        d1, c1 = _data_check_pair(graph, hit[1])
        for _ in range(patience):
            v = pick_vertex.rvs(random_state=rng)
            cand = rng.choice(list(graph.edges(v)))
            d2, c2 = _data_check_pair(graph, cand[:2])
            if d1 != d2 and c1 != c2 and d2 not in graph.neighbors(c1) and d1 not in graph.neighbors(c2):
                graph.remove_edge(d1, c1)
                graph.remove_edge(d2, c2)
                graph.add_edge(d1, c2)
                graph.add_edge(d2, c1)
                break
        else:
            raise RuntimeError("Patience exceeded while selecting an edge to swap in short cycle removal.")
    if not girth_ok():
        raise RuntimeError("Patience exceeded while removing short cycles.")


def code_from_boundary_maps(partial_2, partial_1, compute_logicals=False, check_complex=False) -> QuantumCode:
    """QuantumCode with X checks = partial_2^T and Z checks = partial_1 (the
    chain-complex convention of reference ``homological_product_code.py:90``);
    logicals by GF(2) elimination when asked."""
    x = sp.csr_matrix(sp.csr_matrix(partial_2).T).astype(np.uint32)
    z = sp.csr_matrix(partial_1).astype(np.uint32)
    x.data %= 2
    z.data %= 2
    checks = QuantumCodeChecks(x, z)
    if check_complex and np.any((checks.z @ checks.x.T).toarray() % 2):
        raise AssertionError("boundary maps do not compose to zero")
    if compute_logicals:
        from .gf2 import css_logicals
        lx, lz = css_logicals(checks.x, checks.z)
        if check_complex:
            from .gf2 import rank
            if lx.shape[0] + rank(checks.x.toarray()) + rank(checks.z.toarray()) != checks.num_qubits:
                raise AssertionError("logical count does not match n - rank Hx - rank Hz")
        logicals = QuantumCodeLogicals(lx.astype(np.uint32), lz.astype(np.uint32))
    else:
        logicals = None
    return QuantumCode(checks, logicals)


def homological_product(partial_A, partial_B, check_complex=None, compute_logicals=None) -> QuantumCode:
    """Tensor product of the length-1 complexes A1 -A-> A0 and B1 -B-> B0
    (reference :64-103).

    Qubits are A0xB1 (+) A1xB0; X checks live on A1xB1 and Z checks on A0xB0:
    ``partial_2 = [A (x) I_B1 ; I_A1 (x) B]``, ``partial_1 = [I_A0 (x) B | A (x) I_B0]``."""
    A = sp.csr_matrix(partial_A)
    B = sp.csr_matrix(partial_B)
    (a0, a1), (b0, b1) = A.shape, B.shape
    p2 = sp.vstack([sp.kron(A, sp.identity(b1)), sp.kron(sp.identity(a1), B)]).astype(np.int8)
    p1 = sp.hstack([sp.kron(sp.identity(a0), B), sp.kron(A, sp.identity(b0))]).astype(np.int8)
    assert p2.shape == (a0 * b1 + a1 * b0, a1 * b1) and p1.shape == (a0 * b0, a0 * b1 + a1 * b0)
    return code_from_boundary_maps(p2, p1, compute_logicals=bool(compute_logicals),
                                   check_complex=bool(check_complex))


def biregular_hgp(num_data: int, data_degree: int, check_degree: int, check_complex=None, seed=None,
                  graph_multiedge_retries=None, compute_logicals=None, girth_bound=None,
                  girth_bound_patience=None) -> QuantumCode:
    """Hypergraph product of one random (data_degree, check_degree)-biregular
    Tanner graph with its dual (reference ``hypergraph_product_code.py:7-35``).

    ``biregular_hgp(12, 3, 4, seed=S)`` is the n = 12^2 + 9^2 = 225, k = 9 code of
    the north-star config.  With ``girth_bound`` the classical graph is first
    cleared of cycles of length <= girth_bound (seeded with ``seed + 1``)."""
    nx = _nx()
    num_checks = (num_data * data_degree) // check_degree
    g = random_biregular_graph(num_checks, num_data, data_degree, check_degree, seed=seed,
                               graph_multiedge_retries=graph_multiedge_retries)
    if girth_bound is not None:
        remove_short_cycles(g, girth_bound, seed=None if seed is None else seed + 1,
                            patience=10000 if girth_bound_patience is None else girth_bound_patience)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", FutureWarning)
        data_rows = [v for v in g.nodes if g.nodes[v]["bipartite"] == 0]
        A = nx.bipartite.biadjacency_matrix(g, row_order=data_rows).astype(int)
    code = homological_product(A, A.transpose(), check_complex=check_complex, compute_logicals=compute_logicals)
    assert code.checks.x.shape == code.checks.z.shape
    assert code.num_qubits == num_data ** 2 + num_checks ** 2
    return code


def random_test_hgp(compute_logicals=None) -> QuantumCode:
    """The reference's seeded test code (``hypergraph_product_code.py:37-40``)."""
    return biregular_hgp(36, 3, 4, seed=42, compute_logicals=True if compute_logicals is None else compute_logicals,
                         girth_bound=4)
