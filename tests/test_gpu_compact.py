"""The compact-list path of lean min-sum launches (ms_triage_kernel +
bp_ms_cmp_kernel, qdec_bp_ms.h) against the oracle on the edges the bench
shapes do not reach: every wave shape, batch sizes around the 64-shot triage
tile and the 4-entry chunks, syndrome / readout buffers whose byte length is
not a multiple of 4, more than 64 logicals (several readout-parity words),
no fused check, partial outputs, zero-syndrome shots with and without positive
priors, and the SSF queue carrying readout parities.  Every output equals the
oracle's; the one-pass kernel (QD_OPT_COMPACT = 0) gives the same bytes."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_checks, load_code

pytestmark = pytest.mark.gpu

OUTS = (("iters", "int32"), ("status", "uint8"), ("ssf_steps", "int32"), ("fail", "uint8"))


def _decode_device(dec, syn, rd, keys=("iters", "status", "ssf_steps", "fail")):
    import torch
    dev = torch.device("cuda", 0)
    B = syn.shape[0]
    out = {k: torch.full((B,), 77, dtype=getattr(torch, dt), device=dev) for k, dt in OUTS if k in keys}
    dec.decode_device(B, syn=torch.from_numpy(np.ascontiguousarray(syn)).to(dev),
                      readout=None if rd is None else torch.from_numpy(np.ascontiguousarray(rd)).to(dev), **out)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}, dec.last_kernels()


def _random_graph(rng, m, n, dmax=7, cmax=4):
    from exp_ldpc_amd.codes import make_check_matrix
    rows, colcount = [], np.zeros(n, int)
    for _ in range(m):
        d = int(rng.integers(1, dmax + 1))
        cand = [j for j in rng.permutation(n) if colcount[j] < cmax][:d]
        for j in cand:
            colcount[j] += 1
        rows.append(sorted(cand))
    return make_check_matrix(rows, n)


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("mn", [(40, 90), (110, 170), (120, 230), (100, 370), (200, 520)])
def test_compact_every_wave_shape(gpu_available, oracle_lib, precision, mn, monkeypatch):
    """Random ragged graphs that land on each wave shape; odd m, n (row bytes not
    a multiple of 4); batch sizes 1, 63, 65, 4099; random logicals (k = 3, 70,
    130: one to three parity words); BP only (no SSF)."""
    from exp_ldpc_amd.decoder import Decoder
    m, n = mn
    rng = np.random.default_rng(m * 1000 + n)
    H = _random_graph(rng, m, n)
    probs = rng.uniform(0.005, 0.05, n)
    for k in (3, 70, 130):
        L = (rng.random((k, n)) < 0.05).astype(np.uint8)
        dec = Decoder(H, probs, method="ms", precision=precision, max_iter=20, logicals=L)
        for B in (1, 63, 65, 4099):
            e = (rng.random((B, n)) < 0.02).astype(np.uint8)
            e[: B // 3] = 0
            syn = ((H @ e.T).T % 2).astype(np.uint8)
            rd = (e ^ (rng.random((B, n)) < 0.01)).astype(np.uint8)
            got, (bp_k, _, pre_k) = _decode_device(dec, syn, rd)
            assert "cmp_kernel" in bp_k and "triage" in pre_k, bp_k
            ref = oracle_lib.decode(H, probs, syn, method="ms", precision=precision, max_iter=20, lz=L, readout=rd,
                                    want_llr=False)
            for key in got:
                assert np.array_equal(got[key], ref[key]), (k, B, key)
            dec.set_option("compact", 0)
            one, (bp1, _, _) = _decode_device(dec, syn, rd)
            dec.set_option("compact", 1)
            assert "bp_ms_wave_kernel" in bp1
            for key in got:
                assert np.array_equal(one[key], got[key]), (k, B, key)
            # iteration 1 left to the BP kernel (the triage only lists)
            dec.set_option("triage_it1", 0)
            lst, _ = _decode_device(dec, syn, rd)
            dec.set_option("triage_it1", 1)
            for key in got:
                assert np.array_equal(lst[key], got[key]), (k, B, key)


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_triage_iteration_one_edges(gpu_available, oracle_lib, precision):
    """The triage's iteration-1 tables (it1_tables, qdec_abi.cpp) against the
    oracle where they are most fragile: priors with exact ties between columns
    (the m1 == L_j selection), degree-1 rows (m2 = Big), columns of degree 1..4,
    single-error shots (most converge in iteration 1) next to heavier ones; a
    non-default scaling (tables off) and a negative prior (tables off) give the
    oracle's results too."""
    from exp_ldpc_amd.decoder import Decoder
    rng = np.random.default_rng(77)
    m, n = 96, 150
    H = _random_graph(rng, m, n, dmax=6)
    light = np.flatnonzero(np.diff(sp.csc_matrix(H).indptr) < 4)[[0, 7, 20]]  # room for one more edge
    H = sp.vstack([H, sp.csr_matrix((np.ones(3), ([0, 1, 2], light)), shape=(3, n))]).tocsr()
    levels = np.array([0.01, 0.02, 0.02, 0.04, 0.011])
    probs = levels[rng.integers(0, len(levels), n)]
    B = 2500
    e = np.zeros((B, n), np.uint8)
    e[np.arange(B), rng.integers(0, n, B)] = 1  # one error per shot
    e[B // 2:] |= (rng.random((B - B // 2, n)) < 0.02).astype(np.uint8)
    syn = ((H @ e.T).T % 2).astype(np.uint8)
    rd = (e ^ (rng.random((B, n)) < 0.005)).astype(np.uint8)
    L = (rng.random((5, n)) < 0.1).astype(np.uint8)
    cases = [(probs, 0.0), (probs, 0.625)]
    neg = probs.copy()
    neg[7] = 0.7  # a negative prior LLR
    cases.append((neg, 0.0))
    for pr, scaling in cases:
        dec = Decoder(H, pr, method="ms", precision=precision, max_iter=25, ms_scaling=scaling, logicals=L)
        got, (bp_k, _, pre_k) = _decode_device(dec, syn, rd)
        assert "cmp_kernel" in bp_k and "triage" in pre_k
        ref = oracle_lib.decode(H, pr, syn, method="ms", precision=precision, max_iter=25, ms_scaling=scaling, lz=L,
                                readout=rd, want_llr=False)
        for key in got:
            assert np.array_equal(got[key], ref[key]), (scaling, key)
        if scaling == 0.0 and pr is probs:
            assert (ref["iters"] == 1).mean() > 0.3  # the triage's share is real


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_compact_ssf_rpar_and_partial_outputs(gpu_available, oracle_lib, precision, code225):
    """BP + SSF on the n = 225 code with logicals of 1, 2 and 3 parity words
    (the code's 9 plus random rows): the SSF queue carries readout parities;
    outputs requested in subsets; no readout (no fused check: fail = 0)."""
    from exp_ldpc_amd.decoder import Decoder
    hx, hz = load_checks("hgp_12_3_4_s1234")
    rng = np.random.default_rng(44)
    n = hz.shape[1]
    B = 3001
    e = (rng.random((B, n)) < 0.04).astype(np.uint8)
    e[::7] = 0
    syn = ((hz @ e.T).T % 2).astype(np.uint8)
    rd = (e ^ (rng.random((B, n)) < 0.003)).astype(np.uint8)
    lz9 = code225.logicals.z.toarray() % 2 if sp.issparse(code225.logicals.z) else np.asarray(code225.logicals.z)
    for extra in (0, 60, 140):
        L = np.vstack([lz9, (rng.random((extra, n)) < 0.03).astype(np.uint8)])
        dec = Decoder(hz, 0.027, method="ms", precision=precision, max_iter=30, flip_sets=hx, logicals=L)
        ref = oracle_lib.decode(hz, 0.027, syn, method="ms", precision=precision, max_iter=30, ssf=True, gens=hx, lz=L,
                                readout=rd, want_llr=False, ssf_impl="fast")
        assert ref["ssf_steps"].sum() > 0 and ref["fail"].any()
        # scanning kernel; table-driven kernel behind the queue; SSF fused into
        # the compact BP kernel (QD_OPT_SSF_FUSE, the default: no SSF launch)
        for kern, name, fuse in (("scan", "ssf_wave_kernel", 1), ("auto", "ssf_lut_kernel", 0), ("auto", "", 1)):
            dec.set_option("ssf", kern)
            dec.set_option("ssf_fuse", fuse)
            got, (bp_k, ssf_k, _) = _decode_device(dec, syn, rd)
            assert "cmp_kernel" in bp_k and (name in ssf_k if name else ssf_k == ""), (bp_k, ssf_k)
            for key in got:
                assert np.array_equal(got[key], ref[key]), (extra, kern, key)
        part, _ = _decode_device(dec, syn, rd, keys=("fail",))
        assert np.array_equal(part["fail"], ref["fail"])
        part, _ = _decode_device(dec, syn, rd, keys=("iters", "status"))
        assert np.array_equal(part["iters"], ref["iters"]) and np.array_equal(part["status"], ref["status"])
    nofail, _ = _decode_device(dec, syn, None)
    assert not nofail["fail"].any()
    assert np.array_equal(nofail["iters"], ref["iters"]) and np.array_equal(nofail["status"], ref["status"])


@pytest.mark.parametrize("fuse", [1, 0])
def test_compact_large_batch_counter_tail(gpu_available, oracle_lib, code225, fuse):
    """2^18 shots at p = 0.05 (a compact list long enough for the chunk counter's
    dynamic tail; most BP failures go to SSF, fused into the BP kernel or through
    the queue): a random subset of 3000 shots equals the oracle."""
    import torch
    from exp_ldpc_amd.decoder import Decoder
    hz, hx, lz = code225.checks.z, code225.checks.x, code225.logicals.z
    B, p = 1 << 18, 0.05
    dec = Decoder(hz, 2 * p / 3, method="ms", precision="f64", max_iter=50, flip_sets=hx, logicals=lz)
    dec.set_option("ssf_fuse", fuse)
    dev = torch.device("cuda", 0)
    syn = torch.empty((B, hz.shape[0]), dtype=torch.uint8, device=dev)
    rd = torch.empty((B, hz.shape[1]), dtype=torch.uint8, device=dev)
    dec.sample_storage_device(0, p, p, 3, 0, 0, B, syn, rd)
    out = {k: torch.empty(B, dtype=getattr(torch, dt), device=dev) for k, dt in OUTS}
    dec.decode_device(B, syn=syn, readout=rd, **out)
    torch.cuda.synchronize()
    idx = np.sort(np.random.default_rng(1).choice(B, 3000, replace=False))
    rs, rr = syn.cpu().numpy()[idx], rd.cpu().numpy()[idx]
    ref = oracle_lib.decode(hz, 2 * p / 3, rs, method="ms", precision="f64", max_iter=50, ssf=True, gens=hx, lz=lz,
                            readout=rr, want_llr=False, ssf_impl="fast")
    for k, v in out.items():
        assert np.array_equal(v.cpu().numpy()[idx], ref[k]), k


def test_misaligned_buffers_take_the_one_pass_kernel(gpu_available, oracle_lib, code225):
    """The triage reads 16-B chunks, so syndrome / readout views that do not start
    on a 16-B boundary run the one-pass kernel instead (same results)."""
    import torch
    from exp_ldpc_amd.decoder import Decoder
    hz, hx, lz = code225.checks.z, code225.checks.x, code225.logicals.z
    rng = np.random.default_rng(9)
    B, (m, n) = 777, hz.shape
    e = (rng.random((B, n)) < 0.02).astype(np.uint8)
    syn = ((hz @ e.T).T % 2).astype(np.uint8)
    rd = (e ^ (rng.random((B, n)) < 0.002)).astype(np.uint8)
    dev = torch.device("cuda", 0)
    sbuf = torch.zeros(B * m + 16, dtype=torch.uint8, device=dev)
    rbuf = torch.zeros(B * n + 16, dtype=torch.uint8, device=dev)
    sv = sbuf[3:3 + B * m].view(B, m)
    rv = rbuf[5:5 + B * n].view(B, n)
    sv.copy_(torch.from_numpy(syn))
    rv.copy_(torch.from_numpy(rd))
    dec = Decoder(hz, 0.013, method="ms", precision="f64", max_iter=50, flip_sets=hx, logicals=lz)
    out = {k: torch.empty(B, dtype=getattr(torch, dt), device=dev) for k, dt in OUTS}
    dec.decode_device(B, syn=sv, readout=rv, **out)
    torch.cuda.synchronize()
    assert "bp_ms_wave_kernel" in dec.last_kernels()[0]
    ref = oracle_lib.decode(hz, 0.013, syn, method="ms", precision="f64", max_iter=50, ssf=True, gens=hx, lz=lz,
                            readout=rd, want_llr=False, ssf_impl="fast")
    for k, v in out.items():
        assert np.array_equal(v.cpu().numpy(), ref[k]), k
