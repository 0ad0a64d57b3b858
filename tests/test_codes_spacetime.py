"""Host-side mirrors of the reference's code types, qecc I/O, spacetime
matrices and syndrome helpers, pinned to fixtures generated from the reference
(tests/golden/make_golden.py)."""
import io
import json
import os

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import GOLDEN, load_checks, load_code
from exp_ldpc_amd import gf2
from exp_ldpc_amd.codes import QuantumCode, QuantumCodeChecks, QuantumCodeLogicals, make_check_matrix, \
    read_quantum_code, write_quantum_code
from exp_ldpc_amd.spacetime import SpacetimeCode, SpacetimeCodeSingleShot, spacetime_syndrome, \
    spacetime_syndrome_batch

META = json.load(open(os.path.join(GOLDEN, "golden_meta.json")))
CODES = sorted(META["fixtures"])


@pytest.mark.parametrize("name", CODES)
def test_qecc_roundtrip_matches_reference_writer(name):
    """Reading the reference-written file and writing it back gives the same text."""
    text = open(os.path.join(GOLDEN, f"{name}.qecc")).read()
    code = read_quantum_code(io.StringIO(text), validate_stabilizer_code=True)
    buf = io.StringIO()
    write_quantum_code(buf, code)
    assert buf.getvalue() == text
    hx, hz = load_checks(name)
    assert (code.checks.x != hx).nnz == 0 and (code.checks.z != hz).nnz == 0


@pytest.mark.parametrize("name", CODES)
def test_code_parameters_and_logicals(name):
    meta = META["fixtures"][name]
    code = load_code(name)
    hx, hz = code.checks.x.toarray(), code.checks.z.toarray()
    assert code.num_qubits == meta["n"] and hx.shape[0] == meta["mx"] and hz.shape[0] == meta["mz"]
    assert not ((hx @ hz.T) % 2).any()
    lx, lz = code.logicals.x, code.logicals.z
    assert lz.shape[0] == meta["k"] == code.num_qubits - gf2.rank(hx) - gf2.rank(hz)
    assert not ((hx @ lz.T) % 2).any() and not ((hz @ lx.T) % 2).any()
    assert np.array_equal((lz.astype(int) @ lx.T.astype(int)) % 2, np.eye(lz.shape[0], dtype=int))
    assert gf2.rank(np.vstack([hz, lz])) == gf2.rank(hz) + lz.shape[0]


def test_baseline_code_is_readme_code():
    """README.md:49-50 of the reference: (3,4) HGP on 225 qubits, 108 X and Z checks, 9 logicals."""
    meta = META["fixtures"]["hgp_12_3_4_s1234"]
    assert (meta["n"], meta["mx"], meta["mz"], meta["k"]) == (225, 108, 108, 9)
    hz = load_checks("hgp_12_3_4_s1234")[1]
    assert set(np.asarray(hz.sum(axis=1)).ravel()) == {7}
    assert sorted(np.bincount(np.asarray(hz.sum(axis=0)).ravel())[3:5]) == [81, 144]


def test_reader_errors():
    with pytest.raises(RuntimeError):
        read_quantum_code(io.StringIO("qecc 3 1 1\n0 1 X\n"))
    with pytest.raises(RuntimeError):
        read_quantum_code(io.StringIO("qecc 2 2 1 0\n0 1 X\n0 1 Z\n1 Z\n"))  # overconstrained
    with pytest.raises(RuntimeError):
        read_quantum_code(io.StringIO("qecc 3 1 1 0\n0 5 X\n0 1 Z\n"))  # out of bounds
    with pytest.raises(RuntimeError):
        read_quantum_code(io.StringIO("qecc 3 1 1 0\n0 1 X\n0 2 Z\n"), validate_stabilizer_code=True)


def test_types_and_check_matrix():
    m = make_check_matrix([[0, 2], [1]], 3)
    assert m.toarray().tolist() == [[1, 0, 1], [0, 1, 0]]
    c = QuantumCodeChecks(sp.csr_array(m), m)  # scipy array and matrix flavours both accepted
    assert c.num_qubits == 3 and not c.x.data.flags.writeable
    with pytest.raises(ValueError):
        QuantumCodeChecks(m, make_check_matrix([[0]], 4))
    with pytest.raises(TypeError):
        QuantumCodeChecks(sp.csr_matrix(np.ones((1, 2), dtype=float)), m)
    code = QuantumCode(c)
    assert code.num_logicals == 0


# ---------------------------------------------------------------- spacetime
ST = np.load(os.path.join(GOLDEN, "spacetime_hgp_12_3_4_s1234.npz"))
HZ = load_checks("hgp_12_3_4_s1234")[1]


def _ref_matrix(R):
    return sp.csr_matrix((np.ones(ST[f"R{R}_indices"].size), ST[f"R{R}_indices"], ST[f"R{R}_indptr"]),
                         shape=tuple(ST[f"R{R}_shape"]))


@pytest.mark.parametrize("R", [0, 1, 2, 3])
def test_spacetime_matrix_matches_reference(R):
    mine = SpacetimeCode(HZ, R).spacetime_check_matrix
    ref = _ref_matrix(R)
    assert mine.shape == ref.shape
    assert (sp.csr_matrix(mine) != ref).nnz == 0


@pytest.mark.parametrize("R", [0, 1, 2, 3])
def test_spacetime_syndrome_and_fold_match_reference(R):
    st = SpacetimeCode(HZ, R)
    hist, rd = ST[f"R{R}_history"], ST[f"R{R}_readout"]
    for b in range(hist.shape[0]):
        s = st.syndrome_from_history(lambda t: hist[b, t], rd[b])
        assert np.array_equal(s.astype(np.uint8), ST[f"R{R}_syndrome"][b])
        assert np.array_equal(np.asarray(st.final_correction(ST[f"R{R}_corr"][b])).astype(np.uint8),
                              ST[f"R{R}_fold"][b])
    batch = spacetime_syndrome_batch(R, HZ, hist, rd)
    assert np.array_equal(batch, ST[f"R{R}_syndrome"])
    # reference quirk kept: data_bits boundary at R*r (spacetime_code.py:75)
    prior = np.zeros(st.spacetime_check_matrix.shape[1])
    st.data_bits(prior)[:] = 0.25
    st.measurement_bits(prior)[:] = 0.75
    assert np.array_equal(prior, ST[f"R{R}_prior_split"])


def test_single_shot_matrix():
    ss = SpacetimeCodeSingleShot(HZ)
    H = ss.spacetime_check_matrix.toarray()
    assert H.shape == (108, 333)
    assert np.array_equal(H[:, :225], HZ.toarray()) and np.array_equal(H[:, 225:], np.eye(108))
    x = np.arange(333)
    assert np.array_equal(ss.final_correction(x), x[:225])
