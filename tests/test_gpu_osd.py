"""GPU OSD (qd_osd_batch_device, csrc/qdec_osd.hip) against the host OSD stage
(qd_osd_batch, csrc/qdec_osd.cpp) and the independent numpy checker
(oracle/osd_py.py), bit for bit, on the graphs the decoder modes use: Hz (R=0),
the R=1 spacetime matrix, the single-shot [Hz | I] matrix and a ragged random
code.  Shots BP converged on must be left untouched."""
import zlib

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_checks, load_code

pytestmark = pytest.mark.gpu

HX, HZ = load_checks("hgp_12_3_4_s1234")


def _graphs():
    from exp_ldpc_amd.spacetime import SpacetimeCode, SpacetimeCodeSingleShot
    rng = np.random.default_rng(4)
    m, n = 150, 400
    rows = [sorted(rng.choice(n, size=int(rng.integers(2, 9)), replace=False)) for _ in range(m)]
    from exp_ldpc_amd.codes import make_check_matrix
    return {
        "R0": sp.csr_matrix(HZ),
        "R1": sp.csr_matrix(SpacetimeCode(HZ, 1).spacetime_check_matrix),
        "R2": sp.csr_matrix(SpacetimeCode(HZ, 2).spacetime_check_matrix),
        # beyond the register kernel (m > 384, n >= 1024): workgroup kernel, rows in LDS
        "R3": sp.csr_matrix(SpacetimeCode(HZ, 3).spacetime_check_matrix),
        "R4": sp.csr_matrix(SpacetimeCode(HZ, 4).spacetime_check_matrix),
        "single_shot": sp.csr_matrix(SpacetimeCodeSingleShot(HZ).spacetime_check_matrix),
        "ragged": make_check_matrix(rows, n),
    }


GRAPHS = _graphs()


@pytest.mark.parametrize("gname", list(GRAPHS))
@pytest.mark.parametrize("method,order", [("osd0", 0), ("osd_e", 5), ("osd_cs", 7), ("osd_cs", 0)])
@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_device_osd_matches_host(gpu_available, gname, method, order, precision):
    import torch
    from exp_ldpc_amd.decoder import Decoder
    from exp_ldpc_amd.osd import OsdSolver
    H = GRAPHS[gname]
    m, n = H.shape
    rng = np.random.default_rng(zlib.crc32(f"{gname}/{method}/{order}/{precision}".encode()))
    B = 600
    e = (rng.random((B, n)) < 0.05).astype(np.uint8)
    syn = np.ascontiguousarray((H @ e.T).T % 2, dtype=np.uint8)
    syn[::7] = rng.integers(0, 2, size=syn[::7].shape)  # some arbitrary syndromes too
    dec = Decoder(H, 0.04, method="ms", precision=precision, max_iter=6)
    assert dec.osd_device_supported
    dev = torch.device("cuda", 0)
    syn_d = torch.from_numpy(syn).to(dev)
    tdt = torch.float32 if precision == "f32" else torch.float64
    llr = torch.empty((B, n), dtype=tdt, device=dev)
    status = torch.empty(B, dtype=torch.uint8, device=dev)
    dec.decode_device(B, syn=syn_d, llr=llr, status=status)
    o0 = torch.full((B, n), 0xAA, dtype=torch.uint8, device=dev)
    ow = torch.full((B, n), 0xAA, dtype=torch.uint8, device=dev)
    dec.osd_device(B, llr=llr, method=method, order=order, syn=syn_d, status=status, osd0=o0, osdw=ow)
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    bad = np.nonzero((st & 1) == 0)[0]
    good = np.nonzero(st & 1)[0]
    assert bad.size > 20
    o0h, owh = o0.cpu().numpy(), ow.cpu().numpy()
    assert (o0h[good] == 0xAA).all() and (owh[good] == 0xAA).all()
    r0, rw = OsdSolver(H, method, order).solve(syn[bad], llr.cpu().numpy()[bad].astype(np.float64))
    assert np.array_equal(o0h[bad], r0)
    assert np.array_equal(owh[bad], rw)


def test_device_osd_matches_numpy_checker(gpu_available):
    import torch
    from exp_ldpc_amd.decoder import Decoder
    from oracle.osd_py import osd_decode
    H = GRAPHS["R1"]
    m, n = H.shape
    rng = np.random.default_rng(9)
    B = 64
    e = (rng.random((B, n)) < 0.04).astype(np.uint8)
    syn = np.ascontiguousarray((H @ e.T).T % 2, dtype=np.uint8)
    dec = Decoder(H, 0.03, method="ms", precision="f64", max_iter=3)
    dev = torch.device("cuda", 0)
    syn_d = torch.from_numpy(syn).to(dev)
    llr = torch.empty((B, n), dtype=torch.float64, device=dev)
    ow = torch.zeros((B, n), dtype=torch.uint8, device=dev)
    dec.decode_device(B, syn=syn_d, llr=llr)
    dec.osd_device(B, llr=llr, method="osd_cs", order=7, syn=syn_d, osdw=ow)  # status None: every shot
    torch.cuda.synchronize()
    llr_h, ow_h = llr.cpu().numpy(), ow.cpu().numpy()
    for b in range(0, B, 4):
        _, rw = osd_decode(H, syn[b], llr_h[b], "osd_cs", 7)
        assert np.array_equal(ow_h[b], rw)
        assert ((H @ ow_h[b]) % 2 == syn[b]).all() or not ((H @ rw) % 2 == syn[b]).all()


@pytest.mark.parametrize("mode,rounds", [("bposd", 1), ("bposd", 0), ("bposd", 3), ("bposd_hybrid", 1),
                                         ("bposd_single_shot", 2)])
def test_pipeline_device_osd_equals_host_osd(gpu_available, mode, rounds):
    """The batched pipeline with the device OSD returns the same corrections and
    failure flags as with the host OSD stage (forced by hiding device support)."""
    from exp_ldpc_amd.decoder import Decoder
    from exp_ldpc_amd.experiment import BatchPipeline
    from exp_ldpc_amd.noise_model import depolarizing_noise
    from exp_ldpc_amd.storage_sim import build_storage_simulation
    code = load_code("hgp_12_3_4_s1234")
    opts = {"max_iter": 20, "bp_method": "ms", "ms_scaling_factor": 0, "osd_method": "osd_cs", "osd_order": 7}
    p = 0.03
    sim = build_storage_simulation(rounds, depolarizing_noise(p, p), code)
    pipe = BatchPipeline(code, rounds, mode, opts, (2 * p / 3, 2 * p / 3))
    syn, rd = sim.sample_device(pipe.sampler_graph, 2000, seed=21, stream_id=1)
    dev_res = pipe.run(syn, rd, want_corrections=True)
    orig = Decoder.osd_device_supported
    try:
        Decoder.osd_device_supported = property(lambda self: False)
        host_res = pipe.run(syn, rd, want_corrections=True)
    finally:
        Decoder.osd_device_supported = orig
    assert np.array_equal(dev_res.corrections, host_res.corrections)
    assert np.array_equal(dev_res.fail, host_res.fail)
    assert dev_res.bp_converged < 2000


@pytest.mark.parametrize("gname", ["R3", "R4"])
def test_device_osd_block_matches_numpy_checker(gpu_available, gname):
    """The workgroup OSD kernel (R = 3 / 4 spacetime matrices, rows in LDS)
    against the independent numpy restatement, osd_cs order 7 and osd_e 4."""
    import torch
    from exp_ldpc_amd.decoder import Decoder
    from oracle.osd_py import osd_decode
    H = GRAPHS[gname]
    m, n = H.shape
    assert m > 384 and n >= 1024
    rng = np.random.default_rng(13)
    B = 6
    e = (rng.random((B, n)) < 0.03).astype(np.uint8)
    syn = np.ascontiguousarray((H @ e.T).T % 2, dtype=np.uint8)
    dec = Decoder(H, 0.02, method="ms", precision="f32", max_iter=2)
    assert dec.osd_device_supported
    dev = torch.device("cuda", 0)
    syn_d = torch.from_numpy(syn).to(dev)
    llr = torch.empty((B, n), dtype=torch.float32, device=dev)
    dec.decode_device(B, syn=syn_d, llr=llr)
    for method, order in (("osd_cs", 7), ("osd_e", 4)):
        o0 = torch.zeros((B, n), dtype=torch.uint8, device=dev)
        ow = torch.zeros((B, n), dtype=torch.uint8, device=dev)
        dec.osd_device(B, llr=llr, method=method, order=order, syn=syn_d, osd0=o0, osdw=ow)
        torch.cuda.synchronize()
        llr_h = llr.cpu().numpy().astype(np.float64)
        for b in range(B):
            r0, rw = osd_decode(H, syn[b], llr_h[b], method, order)
            assert np.array_equal(o0.cpu().numpy()[b], r0), (method, b)
            assert np.array_equal(ow.cpu().numpy()[b], rw), (method, b)
            assert ((H @ rw) % 2 == syn[b]).all()
