import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libqdec_hip.so")
    config.addinivalue_line("markers", "slow: long-running")


def load_checks(name):
    d = np.load(os.path.join(GOLDEN, f"{name}_checks.npz"))

    def csr(p):
        return sp.csr_matrix((np.ones(d[p + "_indices"].size, np.uint8), d[p + "_indices"], d[p + "_indptr"]),
                             shape=tuple(d[p + "_shape"]))
    return csr("hx"), csr("hz")


def load_logicals(name):
    """(Lx, Lz) CSR from tests/golden/<name>_logicals.npz."""
    d = np.load(os.path.join(GOLDEN, f"{name}_logicals.npz"))

    def csr(p):
        return sp.csr_matrix((np.ones(d[p + "_indices"].size, np.uint8), d[p + "_indices"], d[p + "_indptr"]),
                             shape=tuple(d[p + "_shape"]))
    return csr("lx"), csr("lz")


def load_code(name):
    from exp_ldpc_amd.codes import read_quantum_code
    with open(os.path.join(GOLDEN, f"{name}.qecc")) as f:
        return read_quantum_code(f, validate_stabilizer_code=True)


@pytest.fixture(scope="session")
def code225():
    return load_code("hgp_12_3_4_s1234")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import load
    return load()


@pytest.fixture(scope="session")
def gpu_available():
    try:
        import torch
        if not torch.cuda.is_available():
            pytest.skip("no GPU")
    except Exception:
        pytest.skip("no torch")
    from exp_ldpc_amd import _abi
    _abi.load()  # fail loudly if the HIP library is missing on a GPU box
    return True
