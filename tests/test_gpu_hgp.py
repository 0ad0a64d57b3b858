"""The hypergraph-product BP kernel (qdec_hgp.cpp / qdec_hgp_kernel.hip,
hipRTC-compiled per code) against the CPU oracle: f64 min-sum, ldpc v1
semantics, hard decisions / iterations / convergence bit-exact."""
import ctypes as C

import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu


def _hgp_decode(dec, syn_dev, B, max_iter, ms_scaling=0.0, slots=0):
    import torch

    from exp_ldpc_amd import _abi
    assert syn_dev.is_contiguous()
    lib = dec._lib
    if slots:
        _abi.check(lib.qd_graph_hgp_set_slots(dec._handle, slots), "hgp slots")
    x = torch.empty((B, dec.n), dtype=torch.uint8, device=syn_dev.device)
    it = torch.empty(B, dtype=torch.int32, device=syn_dev.device)
    st = torch.empty(B, dtype=torch.uint8, device=syn_dev.device)
    _abi.check(lib.qd_graph_hgp_decode_bp(dec._handle, B, syn_dev.data_ptr(), x.data_ptr(), it.data_ptr(),
                                          st.data_ptr(), max_iter, ms_scaling, None), "hgp decode")
    torch.cuda.synchronize()
    return x.cpu().numpy(), it.cpu().numpy(), st.cpu().numpy()


@pytest.mark.parametrize("p", [0.01, 0.05, 0.1])
@pytest.mark.parametrize("slots", [0, 3])
def test_hgp_kernel_bp_parity(gpu_available, oracle_lib, code225, p, slots):
    import torch

    from exp_ldpc_amd.decoder import Decoder
    hz = sp.csr_matrix(code225.checks.z)
    m, n = hz.shape
    rng = np.random.default_rng(int(p * 1000) + slots)
    B = 3000
    e = (rng.random((B, n)) < p).astype(np.uint8)
    syn = np.ascontiguousarray(((hz @ e.T).T % 2).astype(np.uint8))
    prior = 2 * p / 3
    dec = Decoder(hz, prior, method="ms", precision="f64", max_iter=50, device=0)
    info = (C.c_int32 * 8)()
    assert dec._lib.qd_graph_hgp_info(dec._handle, info) == 1
    syn_d = torch.from_numpy(syn).to("cuda:0")
    assert syn_d.is_contiguous()
    x, it, st = _hgp_decode(dec, syn_d, B, 50, slots=slots)
    ref = oracle_lib.decode(hz, prior, syn, method="ms", precision="f64", max_iter=50, want_llr=False)
    assert np.array_equal(it, ref["iters"])
    assert np.array_equal(st & 1, ref["status"] & 1)
    assert np.array_equal(x, ref["x"])
    conv = ref["status"] & 1
    assert 0 < conv.mean() <= 1


def test_hgp_kernel_ms_scaling_and_short_runs(gpu_available, oracle_lib, code225):
    """A fixed scaling factor, max_iter 1 and 2, and a batch that leaves most
    slots of the last workgroups empty."""
    import torch

    from exp_ldpc_amd.decoder import Decoder
    hz = sp.csr_matrix(code225.checks.z)
    rng = np.random.default_rng(7)
    for B, max_iter, scale in ((5, 1, 0.0), (37, 2, 0.625), (700, 30, 0.625)):
        e = (rng.random((B, 225)) < 0.04).astype(np.uint8)
        syn = np.ascontiguousarray(((hz @ e.T).T % 2).astype(np.uint8))
        dec = Decoder(hz, 0.03, method="ms", precision="f64", max_iter=max_iter, ms_scaling=scale, device=0)
        x, it, st = _hgp_decode(dec, torch.from_numpy(syn).to("cuda:0"), B, max_iter, scale)
        ref = oracle_lib.decode(hz, 0.03, syn, method="ms", precision="f64", max_iter=max_iter, ms_scaling=scale,
                                want_llr=False)
        assert np.array_equal(it, ref["iters"]) and np.array_equal(x, ref["x"])
        assert np.array_equal(st & 1, ref["status"] & 1)


def test_hgp_kernel_zero_priors(gpu_available, oracle_lib, code225):
    """Columns with p = 0.5 (prior LLR +0) and p > 0.5: zero and negative
    messages reach the partial states, exercising the kernel's rare exact-parity
    branch and the +0 flag of the merged m2 (MsCore's zero rule)."""
    import torch

    from exp_ldpc_amd.decoder import Decoder
    hz = sp.csr_matrix(code225.checks.z)
    rng = np.random.default_rng(11)
    B = 1000
    e = (rng.random((B, 225)) < 0.03).astype(np.uint8)
    syn = np.ascontiguousarray(((hz @ e.T).T % 2).astype(np.uint8))
    probs = rng.choice([0.5, 0.6, 0.02, 0.02, 0.05], 225)
    dec = Decoder(hz, probs, method="ms", precision="f64", max_iter=25, device=0)
    x, it, st = _hgp_decode(dec, torch.from_numpy(syn).to("cuda:0"), B, 25)
    ref = oracle_lib.decode(hz, probs, syn, method="ms", precision="f64", max_iter=25, want_llr=False)
    assert np.array_equal(it, ref["iters"]) and np.array_equal(x, ref["x"])
    assert np.array_equal(st & 1, ref["status"] & 1)
