"""Noise-model rewrite rules (pinned by the reference's golden test data,
tests/test_storage_sim.py:13-77 of the reference) and the storage-experiment
record views (pinned by views computed with the reference,
tests/golden/storage_views.json)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_code
from exp_ldpc_amd.codes import CircuitTargets
from exp_ldpc_amd.noise_model import circuit_noise, depolarizing_noise, trivial_noise
from exp_ldpc_amd.storage_sim import build_storage_simulation

TOY = ["RX 0 1 2", "TICK", "CZ 0 1", "TICK", "MX 0 2", "TICK", "TICK", "MX 0"]


def test_depolarizing_rewrite_golden():
    got = depolarizing_noise(0.1, 0.2).rewrite(CircuitTargets([1], [0, 2], []), TOY)
    assert list(got) == ["RX 0 1 2", "TICK", "CZ 0 1", "TICK", "DEPOLARIZE1(0.1) 1", "MX(0.2) 0 2", "TICK",
                         "TICK", "DEPOLARIZE1(0.1) 1", "MX(0.2) 0"]


def test_circuit_noise_rewrite_golden():
    got = circuit_noise(0.1, 0.2).rewrite(CircuitTargets([1], [0, 2], []), TOY)
    assert list(got) == ["RX 0 1 2", "DEPOLARIZE1(0.1) 0 1 2", "TICK", "CZ 0 1", "DEPOLARIZE2(0.1) 0 1",
                         "DEPOLARIZE1(0.1) 2", "TICK", "MX(0.2) 0 2", "DEPOLARIZE1(0.1) 0 1 2", "TICK",
                         "DEPOLARIZE1(0.1) 0 1 2", "TICK", "MX(0.2) 0", "DEPOLARIZE1(0.1) 0 1 2"]


def test_trivial_noise_is_identity():
    assert list(trivial_noise().rewrite(CircuitTargets([1], [0, 2], []), TOY)) == TOY


def test_noise_parameters_for_sampler():
    nm = depolarizing_noise(0.03, 0.01)
    assert (nm.kind, nm.p, nm.pm) == ("depolarizing", 0.03, 0.01)


VIEWS = json.load(open(os.path.join(GOLDEN, "storage_views.json")))


@pytest.mark.parametrize("R", [0, 1, 2, 3])
def test_record_views_match_reference(R):
    code = load_code("hgp_12_3_4_s1234")
    sim = build_storage_simulation(R, depolarizing_noise(0.01, 0.01), code, use_x_logicals=False)
    v = VIEWS[str(R)]
    rec = np.arange(v["record_length"])
    for t in range(R):
        assert sim.measurement_view(t, False, rec).tolist() == v["z_rounds"][t]
        assert sim.measurement_view(t, True, rec).tolist() == v["x_rounds"][t]
    assert sim.data_view(rec).tolist() == v["data"]
    # views are views (the reference test checks writes go through)
    sim.data_view(rec)[:] = -1
    assert (rec[v["data"][0]:v["data"][-1] + 1] == -1).all()


@pytest.mark.parametrize("R", [0, 2])
def test_records_from_samples_layout(oracle_lib, R):
    from exp_ldpc_amd.spacetime import SpacetimeCode
    code = load_code("hgp_12_3_4_s1234")
    sim = build_storage_simulation(R, depolarizing_noise(0.05, 0.05), code)
    syn, rd = oracle_lib.sample_storage(code.checks.z, R, 0.05, 0.05, seed=4, stream=0, shot0=0, B=64)
    rec = sim.records_from_samples(syn, rd)
    st = SpacetimeCode(code.checks.z, R)
    for b in range(64):
        hist = lambda t: sim.measurement_view(t, False, rec[b])
        assert np.array_equal(st.syndrome_from_history(hist, sim.data_view(rec[b])).astype(np.uint8), syn[b])
