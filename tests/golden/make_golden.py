"""Generate the golden fixtures under tests/golden/ from the reference itself.

Run in the build container only (needs /root/reference; never on the GPU box):

    python tests/golden/make_golden.py

The reference package imports two third-party modules that are absent from this
image (``galois`` 0.3.5 at ``qecc_util.py:6``; ``stim`` 1.13.0 at
``spacetime_code.py:5``).  To import it, this script writes *throwaway* modules
into a temporary directory outside the repository that only satisfy the imports:
any call into them raises.  Only reference code paths that never touch galois or
stim are executed (code construction without logicals, the ``qecc`` writer/reader,
the spacetime matrices and syndrome helpers, and the storage-circuit text).
Logicals come from this repository's own GF(2) elimination and are validated by
the reference's ``read_quantum_code(validate_stabilizer_code=True)``.

Every output is data (matrices, vectors, circuit text produced by the reference);
no reference source is stored.
"""
from __future__ import annotations

import gzip
import io
import json
import os
import sys
import tempfile

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/python"

_GALOIS_STUB = '''
class FieldArray: pass
class _GFStub:
    def __init__(self, order): self.order = order
    def __call__(self, *a, **k): raise NotImplementedError("galois stub: not available")
def GF(order, *a, **k): return _GFStub(order)
GF2 = GF(2)
class Poly:
    def __init__(self, *a, **k): raise NotImplementedError("galois stub: not available")
'''
_STIM_STUB = '''
class DetectorErrorModel: pass
class Circuit:
    def __init__(self, *a, **k): raise NotImplementedError("stim stub: not available")
'''


def _import_reference():
    stub_dir = tempfile.mkdtemp(prefix="qldpc_stubs_")
    os.makedirs(os.path.join(stub_dir, "galois", "typing"))
    with open(os.path.join(stub_dir, "galois", "__init__.py"), "w") as f:
        f.write(_GALOIS_STUB)
    with open(os.path.join(stub_dir, "galois", "typing", "__init__.py"), "w") as f:
        f.write("ElementLike = object\n")
    with open(os.path.join(stub_dir, "stim.py"), "w") as f:
        f.write(_STIM_STUB)
    sys.dont_write_bytecode = True
    sys.path[:0] = [stub_dir, REF]
    import qldpc  # noqa: F401  (reference)
    import qldpc.spacetime_code as stc
    # scipy >= 1.11 consumes itertools.repeat inside block_diag;
    # give the reference the list it intended so R >= 1 can be generated.
    stc.repeat = lambda x, n: [x] * n
    return qldpc


def _csr_dict(prefix, m):
    m = sp.csr_matrix(m)
    m.sum_duplicates()
    m.sort_indices()
    return {f"{prefix}_indptr": m.indptr.astype(np.int64), f"{prefix}_indices": m.indices.astype(np.int64),
            f"{prefix}_shape": np.array(m.shape, dtype=np.int64)}


def main():
    sys.path.insert(0, REPO)
    from exp_ldpc_amd import gf2  # our own GF(2) elimination

    qldpc = _import_reference()
    from qldpc import biregular_hgp, SpacetimeCode, build_storage_simulation, noise_model
    from qldpc import read_quantum_code as ref_read, write_quantum_code as ref_write
    from qldpc.qecc_util import QuantumCode as RefCode, QuantumCodeLogicals as RefLogicals
    from qldpc.spacetime_code import _spacetime_syndrome

    meta = {"generator": "tests/golden/make_golden.py", "reference_snapshot": "qldpc/exp_ldpc @ 2025-02-21",
            "fixtures": {}}

    codes = {
        # the BASELINE config: scripts/generate_hgp_code.py 4 3 12, seeded
        "hgp_12_3_4_s1234": dict(num_data=12, data_degree=3, check_degree=4, seed=1234),
        # a second seed of the same family (parity-test variety)
        "hgp_12_3_4_s7": dict(num_data=12, data_degree=3, check_degree=4, seed=7),
        # medium code n = 24^2 + 18^2 = 900
        "hgp_24_3_4_s11": dict(num_data=24, data_degree=3, check_degree=4, seed=11),
        # the reference's own test code random_test_hgp (hypergraph_product_code.py:37-40)
        "hgp_36_3_4_s42_g4": dict(num_data=36, data_degree=3, check_degree=4, seed=42, girth_bound=4),
    }
    for name, kw in codes.items():
        code = biregular_hgp(**kw, compute_logicals=False)
        hx, hz = sp.csr_matrix(code.checks.x), sp.csr_matrix(code.checks.z)
        lx, lz = gf2.css_logicals(hx, hz)
        # write through the reference writer, read back through the reference
        # reader with commutation validation
        ref_code = RefCode(code.checks, RefLogicals(lx.astype(np.uint32), lz.astype(np.uint32)))
        buf = io.StringIO()
        ref_write(buf, ref_code)
        text = buf.getvalue()
        back = ref_read(io.StringIO(text), validate_stabilizer_code=True)
        assert (sp.csr_matrix(back.checks.z) != hz).nnz == 0
        with open(os.path.join(HERE, f"{name}.qecc"), "w") as f:
            f.write(text)
        arrs = {}
        arrs.update(_csr_dict("hx", hx))
        arrs.update(_csr_dict("hz", hz))
        np.savez_compressed(os.path.join(HERE, f"{name}_checks.npz"), **arrs)
        meta["fixtures"][name] = {"call": f"biregular_hgp(**{kw}, compute_logicals=False)",
                                  "n": int(hz.shape[1]), "mx": int(hx.shape[0]), "mz": int(hz.shape[0]),
                                  "nnz_z": int(hz.nnz), "k": int(lz.shape[0]),
                                  "rank_hx": gf2.rank(hx.toarray()), "rank_hz": gf2.rank(hz.toarray())}
        print(name, meta["fixtures"][name])

    # ---- spacetime matrices and syndrome/fold pairs on the baseline code ----
    base = np.load(os.path.join(HERE, "hgp_12_3_4_s1234_checks.npz"))
    hz = sp.csr_matrix((np.ones(base["hz_indices"].size, dtype=np.uint32), base["hz_indices"], base["hz_indptr"]),
                       shape=tuple(base["hz_shape"]))
    r, n = hz.shape
    rng = np.random.default_rng(20250221)
    st_arrays = {}
    for R in (0, 1, 2, 3):
        stc = SpacetimeCode(hz, R)
        H = sp.csr_matrix(stc.spacetime_check_matrix)
        st_arrays.update(_csr_dict(f"R{R}", H))
        B = 16
        hist = rng.integers(0, 2, size=(B, R, r)).astype(np.uint8)
        rd = rng.integers(0, 2, size=(B, n)).astype(np.uint8)
        syn = np.stack([stc.syndrome_from_history(lambda t, h=hist[b]: h[t], rd[b]) for b in range(B)])
        syn2 = np.stack([_spacetime_syndrome(R, hz, lambda t, h=hist[b]: h[t], rd[b]) for b in range(B)])
        assert np.array_equal(syn, syn2)
        corr = rng.integers(0, 2, size=(B, H.shape[1])).astype(np.uint8)
        fold = np.stack([stc.final_correction(corr[b]) for b in range(B)])
        st_arrays[f"R{R}_history"] = hist
        st_arrays[f"R{R}_readout"] = rd
        st_arrays[f"R{R}_syndrome"] = syn.astype(np.uint8)
        st_arrays[f"R{R}_corr"] = corr
        st_arrays[f"R{R}_fold"] = np.asarray(fold).astype(np.uint8)
        prior = np.zeros(H.shape[1])
        stc.data_bits(prior)[:] = 0.25
        stc.measurement_bits(prior)[:] = 0.75
        st_arrays[f"R{R}_prior_split"] = prior
    np.savez_compressed(os.path.join(HERE, "spacetime_hgp_12_3_4_s1234.npz"), **st_arrays)

    # ---- storage experiment circuits (depolarizing_noise(p, pm=p)) ----
    ref_code = ref_read(open(os.path.join(HERE, "hgp_12_3_4_s1234.qecc")), validate_stabilizer_code=True)
    views = {}
    for R in (0, 1, 2, 3):
        sim = build_storage_simulation(R, noise_model.depolarizing_noise(0.01, 0.01), ref_code, use_x_logicals=False)
        with gzip.open(os.path.join(HERE, f"storage_R{R}.txt.gz"), "wt") as f:
            f.write("\n".join(sim.circuit))
        rec_len = (hz.shape[0] * 2) * R + n
        vec = np.arange(rec_len)
        views[str(R)] = {
            "record_length": rec_len,
            "z_rounds": [sim.measurement_view(t, False, vec).tolist() for t in range(R)],
            "x_rounds": [sim.measurement_view(t, True, vec).tolist() for t in range(R)],
            "data": sim.data_view(vec).tolist(),
        }
    with open(os.path.join(HERE, "storage_views.json"), "w") as f:
        json.dump(views, f)

    with open(os.path.join(HERE, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("done")


GRAPH_SEEDS = [0x59824c5a, 0x9dca707a, 0xe0218aa8, 0x81da8035]  # first seeds of tests/test_random_biregular_graph.py:21
GRAPH_SHAPES = [(27, 3, 4), (10, 5, 6), (21, 7, 8), (27, 9, 10)]   # (left vertices, right degree, left degree), :28-33


def graphs():
    """Edge lists of the reference's random_biregular_graph / remove_short_cycles on
    the shapes its own tests use, plus the C4 code (biregular_hgp(80,3,4), n=10^4)
    checks.  Output: graphs.npz, hgp_80_3_4_s2025_checks.npz."""
    sys.path.insert(0, REPO)
    _import_reference()
    from qldpc import biregular_hgp, random_biregular_graph, remove_short_cycles
    out = {}
    for (lv, rdeg, ldeg) in GRAPH_SHAPES:
        for s in GRAPH_SEEDS:
            g = random_biregular_graph(lv, lv * ldeg // rdeg, rdeg, ldeg, seed=s)
            out[f"rbg_{lv}_{rdeg}_{ldeg}_{s}"] = np.array(sorted((min(u, v), max(u, v)) for u, v in g.edges()),
                                                          dtype=np.int64)
    for s in GRAPH_SEEDS[:2]:  # tests/test_random_biregular_graph.py:41-53
        g = random_biregular_graph(102, 102 * 4 // 3, 3, 4, seed=s)
        remove_short_cycles(g, 4, seed=s - 42, patience=10000)
        out[f"girth4_102_3_4_{s}"] = np.array(sorted((min(u, v), max(u, v)) for u, v in g.edges()), dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "graphs.npz"), **out)
    code = biregular_hgp(80, 3, 4, seed=2025, compute_logicals=False)
    arrs = {}
    arrs.update(_csr_dict("hx", code.checks.x))
    arrs.update(_csr_dict("hz", code.checks.z))
    np.savez_compressed(os.path.join(HERE, "hgp_80_3_4_s2025_checks.npz"), **arrs)
    print("graphs done:", len(out), "graphs; C4 code", code.checks.z.shape, code.checks.z.nnz)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--graphs":
        graphs()
    else:
        main()
