"""GPU parity: the HIP decoder (through the C ABI) against the CPU oracle on the
same seeded inputs.  Bar: bit-exact hard decisions, iteration counts, status,
SSF steps, corrections and failure flags; min-sum LLRs bit-exact; product-sum
LLRs (ldpc's log(1/ratio) output, computed with the device log) within
rtol 1e-12 (f64) / 1e-6 (f32)."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_checks, load_code

pytestmark = pytest.mark.gpu

HX, HZ = load_checks("hgp_12_3_4_s1234")


def _errors(rng, B, n, p):
    return (rng.random((B, n)) < p).astype(np.uint8)


def _spacetime(R):
    from exp_ldpc_amd.spacetime import SpacetimeCode
    return SpacetimeCode(HZ, R).spacetime_check_matrix


def _cmp_llr(a, b, method, precision):
    if method == "ms":
        assert np.array_equal(a.astype(np.float64), b), "min-sum LLRs must be bit-exact"
    else:
        rtol = 1e-12 if precision == "f64" else 1e-6
        a = a.astype(np.float64)
        fin = np.isfinite(b)
        assert np.array_equal(np.isfinite(a), fin)
        assert np.array_equal(a[~fin], b[~fin])
        np.testing.assert_allclose(a[fin], b[fin], rtol=rtol, atol=0)


@pytest.mark.parametrize("method", ["ms", "ps"])
@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("shape", ["R0", "R1"])
def test_bp_parity(gpu_available, oracle_lib, method, precision, shape):
    from exp_ldpc_amd.decoder import Decoder
    H = HZ if shape == "R0" else _spacetime(1)
    m, n = H.shape
    rng = np.random.default_rng(hash((method, precision, shape)) % 2**32)
    B = 3000
    p = np.where(rng.random(B) < 0.5, 0.01, 0.04)[:, None]
    e = (rng.random((B, n)) < p).astype(np.uint8)
    syn = ((sp.csr_matrix(H) @ e.T).T % 2).astype(np.uint8)
    prior = 0.02
    dec = Decoder(H, prior, method=method, precision=precision, max_iter=40)
    got = dec.decode(syn, want=("x", "llr", "iters", "status"))
    ref = oracle_lib.decode(H, prior, syn, method=method, precision=precision, max_iter=40)
    assert np.array_equal(got["iters"], ref["iters"])
    assert np.array_equal(got["status"], ref["status"])
    assert np.array_equal(got["x"], ref["x"])
    _cmp_llr(got["llr"], ref["llr"], method, precision)
    # both converged and non-converged shots are exercised
    conv = ref["status"] & 1
    assert 0 < conv.mean() < 1


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("max_iter", [1, 3, 50])
@pytest.mark.parametrize("ssf_kernel", ["auto", "scan", "scan_gather", "scan_nosplit"])
def test_bp_ssf_parity(gpu_available, oracle_lib, precision, max_iter, ssf_kernel, code225):
    """Every wave SSF kernel against the oracle: the table-driven kernel (the
    default on this code: one score table for all 108 generators), and the
    scanning kernel with its local syndromes updated through the check ->
    generator table after each flip, re-gathered from the residual every step,
    or scored one lane per generator (QD_OPT_SSF)."""
    from exp_ldpc_amd.decoder import Decoder
    rng = np.random.default_rng(max_iter)
    B = 2000
    rd = _errors(rng, B, 225, 0.03)
    syn = ((HZ @ rd.T).T % 2).astype(np.uint8)
    lz = code225.logicals.z
    dec = Decoder(HZ, 0.02, method="ms", precision=precision, max_iter=max_iter, flip_sets=HX, logicals=lz)
    dec.set_option("ssf", ssf_kernel)
    assert dec.ssf_tables()[0]
    got = dec.decode(syn, readout=rd, want=("x", "corr", "iters", "status", "ssf_steps", "fail"))
    assert ("ssf_lut_kernel" if ssf_kernel == "auto" else "ssf_wave_kernel") in dec.last_kernels()[1]
    ref = oracle_lib.decode(HZ, 0.02, syn, method="ms", precision=precision, max_iter=max_iter, ssf=True, gens=HX,
                            lz=lz, readout=rd, want_llr=False)
    for key in ("x", "corr", "iters", "status", "ssf_steps", "fail"):
        assert np.array_equal(got[key], ref[key]), key
    assert ref["ssf_steps"].sum() > 0


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("ssf_kernel", ["auto", "scan"])
def test_bp_ssf_parity_long_queue(gpu_available, oracle_lib, precision, ssf_kernel, code225):
    """A queue long enough (2^18 BP failures, >= 16 slots per SSF wave) that the
    SSF kernel hands out its tail from the slot counter; shots are independent,
    so a random subset decoded by the oracle checks every output bit-exactly."""
    from exp_ldpc_amd.decoder import Decoder
    rng = np.random.default_rng(18)
    B = 1 << 18
    rd = _errors(rng, B, 225, 0.08)
    syn = ((HZ @ rd.T).T % 2).astype(np.uint8)
    lz = code225.logicals.z
    dec = Decoder(HZ, 0.05, method="ms", precision=precision, max_iter=2, flip_sets=HX, logicals=lz)
    dec.set_option("ssf", ssf_kernel)
    got = dec.decode(syn, readout=rd, want=("x", "corr", "iters", "status", "ssf_steps", "fail"))
    assert ("ssf_lut_kernel" if ssf_kernel == "auto" else "ssf_wave_kernel") in dec.last_kernels()[1]
    assert (got["status"] & 1).mean() < 0.05  # nearly every shot went to the SSF queue
    idx = np.sort(rng.choice(B, 3000, replace=False))  # ~600 of them from counter-handed slots
    ref = oracle_lib.decode(HZ, 0.05, syn[idx], method="ms", precision=precision, max_iter=2, ssf=True, gens=HX,
                            lz=lz, readout=rd[idx], want_llr=False)
    for key in ("x", "corr", "iters", "status", "ssf_steps", "fail"):
        assert np.array_equal(got[key][idx], ref[key]), key
    assert ref["ssf_steps"].mean() > 5


def test_ssf_bounded_steps(gpu_available, oracle_lib):
    from exp_ldpc_amd.decoder import Decoder
    rng = np.random.default_rng(5)
    rd = _errors(rng, 500, 225, 0.06)
    syn = ((HZ @ rd.T).T % 2).astype(np.uint8)
    for steps in (1, 2):
        dec = Decoder(HZ, 0.03, method="ms", precision="f32", max_iter=2, flip_sets=HX, ssf_max_steps=steps)
        got = dec.decode(syn, want=("x", "ssf_steps", "status"))
        ref = oracle_lib.decode(HZ, 0.03, syn, method="ms", precision="f32", max_iter=2, ssf=True, gens=HX,
                                ssf_max_steps=steps, want_llr=False)
        assert got["ssf_steps"].max() <= steps
        for key in ("x", "ssf_steps", "status"):
            assert np.array_equal(got[key], ref[key]), key


def test_spacetime_fold_and_fail(gpu_available, oracle_lib, code225):
    """R=1 spacetime decode with the fused fold (SpacetimeCode.final_correction)
    and failure flag."""
    from exp_ldpc_amd.decoder import Decoder
    H = _spacetime(1)
    syn, rd = oracle_lib.sample_storage(HZ, 1, 0.02, 0.02, seed=3, stream=0, shot0=0, B=3000)
    lz = code225.logicals.z
    dec = Decoder(H, 2 * 0.02 / 3, method="ms", precision="f32", max_iter=30, n_data=225, fold_blocks=2, logicals=lz)
    got = dec.decode(syn, readout=rd, want=("x", "corr", "iters", "status", "fail"))
    ref = oracle_lib.decode(H, 2 * 0.02 / 3, syn, method="ms", precision="f32", max_iter=30, n_data=225,
                            fold_blocks=2, lz=lz, readout=rd, want_llr=False)
    for key in ("x", "corr", "iters", "status", "fail"):
        assert np.array_equal(got[key], ref[key]), key
    fold = (ref["x"][:, :225] ^ ref["x"][:, 225:450])
    assert np.array_equal(got["corr"], fold)


def test_hybrid_stage2_syndrome_from_vectors(gpu_available, oracle_lib, code225):
    """bpssf_hybrid stage 2: syndrome = Hz (readout ^ stage-1 correction)."""
    from exp_ldpc_amd.decoder import Decoder
    rng = np.random.default_rng(11)
    B = 1500
    rd = _errors(rng, B, 225, 0.03)
    c1 = _errors(rng, B, 225, 0.01)
    lz = code225.logicals.z
    dec = Decoder(HZ, 0.02, method="ms", precision="f32", max_iter=20, flip_sets=HX, logicals=lz)
    got = dec.decode(None, base=c1, readout=rd, syn_flags=3, want=("x", "corr", "iters", "status", "ssf_steps", "fail"))
    ref = oracle_lib.decode(HZ, 0.02, None, method="ms", precision="f32", max_iter=20, ssf=True, gens=HX, lz=lz,
                            base=c1, readout=rd, syn_flags=3, B=B, want_llr=False)
    for key in ("x", "corr", "iters", "status", "ssf_steps", "fail"):
        assert np.array_equal(got[key], ref[key]), key


@pytest.mark.parametrize("rounds", [0, 1, 2, 3])
def test_sampler_parity(gpu_available, oracle_lib, rounds):
    import torch
    from exp_ldpc_amd.decoder import Decoder
    dec = Decoder(HZ, 0.01)
    B, shot0 = 4000, 12345
    m, n = HZ.shape
    syn = torch.empty((B, (rounds + 1) * m), dtype=torch.uint8, device="cuda")
    rd = torch.empty((B, n), dtype=torch.uint8, device="cuda")
    dec.sample_storage_device(rounds, 0.03, 0.02, seed=20250221, stream_id=4, shot0=shot0, B=B, syn=syn, readout=rd)
    torch.cuda.synchronize()
    rs, rr = oracle_lib.sample_storage(HZ, rounds, 0.03, 0.02, seed=20250221, stream=4, shot0=shot0, B=B)
    assert np.array_equal(syn.cpu().numpy(), rs)
    assert np.array_equal(rd.cpu().numpy(), rr)
    # sharding invariance: the second half sampled alone equals the tail
    syn2 = torch.empty((B // 2, (rounds + 1) * m), dtype=torch.uint8, device="cuda")
    rd2 = torch.empty((B // 2, n), dtype=torch.uint8, device="cuda")
    dec.sample_storage_device(rounds, 0.03, 0.02, seed=20250221, stream_id=4, shot0=shot0 + B // 2, B=B // 2,
                              syn=syn2, readout=rd2)
    torch.cuda.synchronize()
    assert np.array_equal(syn2.cpu().numpy(), rs[B // 2:])


def test_edge_cases(gpu_available, oracle_lib):
    from exp_ldpc_amd.decoder import Decoder
    dec = Decoder(HZ, 0.01, method="ms", precision="f32", max_iter=0, flip_sets=HX)
    # all-zero syndrome: trivial decode converges at iteration 1 (no ldpc shortcut)
    z = np.zeros((3, HZ.shape[0]), np.uint8)
    out = dec.decode(z, want=("x", "iters", "status"))
    assert not out["x"].any() and (out["iters"] == 1).all() and (out["status"] == 3).all()
    # single shot, max_iter = 0 -> n
    rng = np.random.default_rng(2)
    s = rng.integers(0, 2, (1, HZ.shape[0])).astype(np.uint8)
    got = dec.decode(s, want=("x", "iters", "status", "ssf_steps"))
    ref = oracle_lib.decode(HZ, 0.01, s, method="ms", precision="f32", max_iter=0, ssf=True, gens=HX, want_llr=False)
    for key in ("x", "iters", "status", "ssf_steps"):
        assert np.array_equal(got[key], ref[key]), key


@pytest.mark.parametrize("seed", [1, 2])
def test_random_irregular_codes(gpu_available, oracle_lib, seed):
    """Ragged degrees (1..8 per check, 0..4 per variable), odd sizes."""
    from exp_ldpc_amd.decoder import Decoder
    rng = np.random.default_rng(seed)
    m, n = int(rng.integers(20, 200)), int(rng.integers(30, 500))
    rows = []
    colcount = np.zeros(n, int)
    for i in range(m):
        d = int(rng.integers(1, 9))
        cand = [j for j in rng.permutation(n) if colcount[j] < 4][:d]
        for j in cand:
            colcount[j] += 1
        rows.append(sorted(cand))
    from exp_ldpc_amd.codes import make_check_matrix
    H = make_check_matrix(rows, n)
    e = _errors(rng, 1000, n, 0.03)
    syn = ((H @ e.T).T % 2).astype(np.uint8)
    probs = rng.uniform(0.005, 0.1, n)
    for method in ("ms", "ps"):
        for precision in ("f32", "f64"):
            dec = Decoder(H, probs, method=method, precision=precision, max_iter=25)
            got = dec.decode(syn, want=("x", "llr", "iters", "status"))
            ref = oracle_lib.decode(H, probs, syn, method=method, precision=precision, max_iter=25)
            for key in ("x", "iters", "status"):
                assert np.array_equal(got[key], ref[key]), (method, precision, key)
            _cmp_llr(got["llr"], ref["llr"], method, precision)


def _graph(name):
    from exp_ldpc_amd.spacetime import SpacetimeCode
    if name.startswith("st"):  # st<R>_<code>
        R, code = name[2], name[4:]
        return SpacetimeCode(load_checks(code)[1], int(R)).spacetime_check_matrix, None
    hx, hz = load_checks(name)
    return hz, hx


BLOCK_GRAPHS = ["hgp_24_3_4_s11", "hgp_36_3_4_s42_g4", "st2_hgp_12_3_4_s1234", "st3_hgp_12_3_4_s1234",
                "st1_hgp_36_3_4_s42_g4"]


@pytest.mark.parametrize("name", BLOCK_GRAPHS)
@pytest.mark.parametrize("method,precision", [("ms", "f32"), ("ps", "f32"), ("ps", "f64"), ("ms", "f64")])
def test_block_kernel_parity(gpu_available, oracle_lib, name, method, precision):
    """Graphs outside the wave shapes (n > 576, row degree 9 at R >= 2, HBM
    message scratch for the 36x36 spacetime graph) take the workgroup kernels."""
    from exp_ldpc_amd.decoder import Decoder
    H, _ = _graph(name)
    H = sp.csr_matrix(H)
    rng = np.random.default_rng(len(name))
    B = 300
    e = (rng.random((B, H.shape[1])) < 0.02).astype(np.uint8)
    syn = ((H @ e.T).T % 2).astype(np.uint8)
    dec = Decoder(H, 0.015, method=method, precision=precision, max_iter=25)
    got = dec.decode(syn, want=("x", "llr", "iters", "status"))
    ref = oracle_lib.decode(H, 0.015, syn, method=method, precision=precision, max_iter=25)
    for key in ("x", "iters", "status"):
        assert np.array_equal(got[key], ref[key]), key
    _cmp_llr(got["llr"], ref["llr"], method, precision)


@pytest.mark.parametrize("name", ["hgp_24_3_4_s11", "hgp_36_3_4_s42_g4"])
def test_block_ssf_parity(gpu_available, oracle_lib, name):
    from conftest import load_code
    from exp_ldpc_amd.decoder import Decoder
    code = load_code(name)
    hx, hz = code.checks.x, code.checks.z
    rng = np.random.default_rng(5)
    B = 400
    rd = (rng.random((B, hz.shape[1])) < 0.03).astype(np.uint8)
    syn = ((hz @ rd.T).T % 2).astype(np.uint8)
    dec = Decoder(hz, 0.02, method="ms", precision="f32", max_iter=8, flip_sets=hx, logicals=code.logicals.z)
    got = dec.decode(syn, readout=rd, want=("x", "corr", "iters", "status", "ssf_steps", "fail"))
    ref = oracle_lib.decode(hz, 0.02, syn, method="ms", precision="f32", max_iter=8, ssf=True, gens=hx,
                            lz=code.logicals.z, readout=rd, want_llr=False, ssf_impl="fast")
    for key in ("x", "corr", "iters", "status", "ssf_steps", "fail"):
        assert np.array_equal(got[key], ref[key]), key
    assert ref["ssf_steps"].sum() > 0


def test_spacetime_r2_fold(gpu_available, oracle_lib, code225):
    from exp_ldpc_amd.decoder import Decoder
    H = _spacetime(2)
    syn, rd = oracle_lib.sample_storage(HZ, 2, 0.01, 0.01, seed=8, stream=0, shot0=0, B=800)
    lz = code225.logicals.z
    dec = Decoder(H, 0.0067, method="ms", precision="f32", max_iter=30, n_data=225, fold_blocks=3, logicals=lz)
    got = dec.decode(syn, readout=rd, want=("corr", "iters", "status", "fail"))
    ref = oracle_lib.decode(H, 0.0067, syn, method="ms", precision="f32", max_iter=30, n_data=225, fold_blocks=3,
                            lz=lz, readout=rd, want_llr=False)
    for key in ("corr", "iters", "status", "fail"):
        assert np.array_equal(got[key], ref[key]), key


def test_kernel_timing_ring(gpu_available, oracle_lib, code225):
    """qd_graph_set_timing/read_timing: one (BP, SSF) duration pair per decode
    call up to the capacity; results unchanged by timing."""
    from exp_ldpc_amd.decoder import Decoder
    rng = np.random.default_rng(77)
    rd = _errors(rng, 4000, 225, 0.04)
    syn = ((HZ @ rd.T).T % 2).astype(np.uint8)
    dec = Decoder(HZ, 0.03, method="ms", precision="f32", max_iter=30, flip_sets=HX, logicals=code225.logicals.z)
    base = dec.decode(syn, readout=rd, want=("x", "fail"))
    dec.set_timing(2)
    outs = [dec.decode(syn, readout=rd, want=("x", "fail")) for _ in range(3)]
    bp, ssf = dec.read_timing()
    assert bp.shape == (2,) and ssf.shape == (2,)
    assert (bp > 0).all() and (ssf > 0).all()
    for o in outs:
        assert np.array_equal(o["x"], base["x"]) and np.array_equal(o["fail"], base["fail"])
    assert dec.read_timing()[0].shape == (0,)
    dec.set_timing(0)
    dec.decode(syn, readout=rd, want=("fail",))


@pytest.mark.parametrize("packed", [False, True])
def test_split_ssf_back_to_back_on_one_handle(gpu_available, oracle_lib, packed):
    """Split SSF (qd_graph_set_ssf_stream) with its double-buffered queues: five
    decodes on ONE handle enqueued back to back on one BP stream, their SSF
    kernels on a second stream (decode k's BP overlaps decode k-1's SSF; decode
    k waits only for decode k-2's SSF).  Every output equals the oracle."""
    import torch
    from exp_ldpc_amd.decoder import Decoder, pack_rows
    dev = torch.device("cuda", 0)
    p, B, K = 0.06, 4096, 5
    lz = np.asarray(load_code("hgp_12_3_4_s1234").logicals.z) % 2
    syn, rd = oracle_lib.sample_storage(HZ, 0, p, p, seed=21, stream=1, shot0=0, B=K * B)
    ref = oracle_lib.decode(HZ, 2 * p / 3, syn, method="ms", precision="f64", max_iter=50, ssf=True, gens=HX,
                            lz=lz, readout=rd, want_llr=False, ssf_impl="fast")
    dec = Decoder(HZ, 2 * p / 3, method="ms", precision="f64", max_iter=50, flip_sets=HX, logicals=lz)
    if packed:
        syn_d = torch.from_numpy(pack_rows(syn).view(np.int64)).to(dev)
        rd_d = torch.from_numpy(pack_rows(rd).view(np.int64)).to(dev)
    else:
        syn_d, rd_d = torch.from_numpy(syn).to(dev), torch.from_numpy(rd).to(dev)
    outs = {k: torch.full((K * B,), 7, dtype=dt, device=dev) for k, dt in
            (("iters", torch.int32), ("status", torch.uint8), ("ssf_steps", torch.int32), ("fail", torch.uint8))}
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    dec.set_ssf_stream(s2)
    for k in range(K):
        sl = slice(k * B, (k + 1) * B)
        dec.decode_device(B, syn=syn_d[sl], readout=rd_d[sl], stream=s1.cuda_stream, packed=packed,
                          **{n: v[sl] for n, v in outs.items()})
    torch.cuda.synchronize()
    dec.set_ssf_stream(None)
    assert dec.last_kernels()[1]  # an SSF kernel ran
    for n, v in outs.items():
        assert np.array_equal(v.cpu().numpy(), ref[n]), n
    assert ref["ssf_steps"].sum() > 0


def test_ssf_stream_split_and_handle_chain(gpu_available, oracle_lib):
    """qd_graph_set_ssf_stream: BP on one stream, SSF on another behind an event;
    then two decodes on ONE handle enqueued on two different streams back to back
    (the handle's workspace chain orders them).  Every output equals the oracle."""
    import torch
    from exp_ldpc_amd.decoder import Decoder
    dev = torch.device("cuda", 0)
    p = 0.05
    B = 3000
    lz = np.asarray(load_code("hgp_12_3_4_s1234").logicals.z) % 2
    syn, rd = oracle_lib.sample_storage(HZ, 0, p, p, seed=9, stream=0, shot0=0, B=2 * B)
    ref = oracle_lib.decode(HZ, 2 * p / 3, syn, method="ms", precision="f64", max_iter=50, ssf=True, gens=HX,
                            lz=lz, readout=rd, want_llr=False, ssf_impl="fast")
    dec = Decoder(HZ, 2 * p / 3, method="ms", precision="f64", max_iter=50, flip_sets=HX, logicals=lz)
    s1, s2, s3 = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    outs = []
    syn_d, rd_d = torch.from_numpy(syn).to(dev), torch.from_numpy(rd).to(dev)
    for _ in range(2):
        outs.append({k: torch.empty(B, dtype=dt, device=dev) for k, dt in
                     (("iters", torch.int32), ("status", torch.uint8), ("ssf_steps", torch.int32),
                      ("fail", torch.uint8))})
    torch.cuda.synchronize()  # inputs are on the device before the side streams read them
    dec.set_ssf_stream(s3)
    for h, st in ((0, s1), (1, s2)):
        sl = slice(h * B, (h + 1) * B)
        dec.decode_device(B, syn=syn_d[sl], readout=rd_d[sl], stream=st.cuda_stream, **outs[h])
    torch.cuda.synchronize()
    dec.set_ssf_stream(None)
    for h in (0, 1):
        sl = slice(h * B, (h + 1) * B)
        for k in ("iters", "status", "ssf_steps", "fail"):
            assert np.array_equal(outs[h][k].cpu().numpy(), ref[k][sl]), (h, k)


def test_empty_batch_and_buffer_validation(gpu_available):
    """B = 0 is a no-op on every entry point; mistyped or short device buffers
    are rejected in Python before any launch (no out-of-bounds device access)."""
    import torch
    from exp_ldpc_amd.decoder import Decoder
    dev = torch.device("cuda", 0)
    dec = Decoder(HZ, 0.01, method="ms", precision="f64", max_iter=10, flip_sets=HX)
    out = dec.decode(np.zeros((0, HZ.shape[0]), np.uint8))
    assert out["x"].shape == (0, HZ.shape[1]) and out["fail"].shape == (0,)
    e = torch.empty((0, HZ.shape[0]), dtype=torch.uint8, device=dev)
    dec.decode_device(0, syn=e, iters=torch.empty(0, dtype=torch.int32, device=dev))
    dec.sample_storage_device(0, 0.01, 0.01, 1, 0, 0, 0, e, torch.empty((0, HZ.shape[1]), dtype=torch.uint8,
                                                                         device=dev))
    llr = torch.empty((0, HZ.shape[1]), dtype=torch.float64, device=dev)
    dec.osd_device(0, llr=llr, method="osd_cs", order=7, syn=e)
    torch.cuda.synchronize()
    B = 8
    syn = torch.zeros((B, HZ.shape[0]), dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError):  # f32 llr buffer for an f64 decoder
        dec.decode_device(B, syn=syn, llr=torch.empty((B, HZ.shape[1]), dtype=torch.float32, device=dev))
    with pytest.raises(ValueError):  # too short
        dec.decode_device(B, syn=syn[:4])
    with pytest.raises(ValueError):  # host tensor
        dec.decode_device(B, syn=syn.cpu())


@pytest.mark.parametrize("name", BLOCK_GRAPHS)
def test_lds_kernel_block_graphs(gpu_available, oracle_lib, name, monkeypatch):
    """bp_ms_lds_kernel forced (QD_OPT_LDS_KERNEL = 1) on the workgroup-kernel graphs,
    min-sum f32 (its only configuration): x / iterations / status bit-exact."""
    from exp_ldpc_amd.decoder import Decoder
    from exp_ldpc_amd import decoder
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "lds_kernel", 1)
    H, _ = _graph(name)
    H = sp.csr_matrix(H)
    rng = np.random.default_rng(len(name) + 1)
    B = 300
    e = (rng.random((B, H.shape[1])) < 0.02).astype(np.uint8)
    syn = ((H @ e.T).T % 2).astype(np.uint8)
    dec = Decoder(H, 0.015, method="ms", precision="f32", max_iter=25)
    got = dec.decode(syn, want=("x", "iters", "status"))
    ref = oracle_lib.decode(H, 0.015, syn, method="ms", precision="f32", max_iter=25)
    for key in ("x", "iters", "status"):
        assert np.array_equal(got[key], ref[key]), key


def test_lds_kernel_ssf_fold(gpu_available, oracle_lib, code225, monkeypatch):
    """bp_ms_lds_kernel + the incremental SSF block kernel forced on a block graph
    with flip sets and logicals, and on the R = 2 spacetime graph with the fold
    onto the data qubits (fold_blocks = 3) and the fused logical check."""
    from conftest import load_code
    from exp_ldpc_amd.decoder import Decoder
    from exp_ldpc_amd import decoder
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "lds_kernel", 1)
    code = load_code("hgp_36_3_4_s42_g4")
    hx, hz = code.checks.x, code.checks.z
    rng = np.random.default_rng(9)
    rd = (rng.random((400, hz.shape[1])) < 0.03).astype(np.uint8)
    syn = ((hz @ rd.T).T % 2).astype(np.uint8)
    dec = Decoder(hz, 0.02, method="ms", precision="f32", max_iter=12, flip_sets=hx, logicals=code.logicals.z)
    keys = ("x", "corr", "iters", "status", "ssf_steps", "fail")
    got = dec.decode(syn, readout=rd, want=keys)
    ref = oracle_lib.decode(hz, 0.02, syn, method="ms", precision="f32", max_iter=12, ssf=True, gens=hx,
                            lz=code.logicals.z, readout=rd, want_llr=False, ssf_impl="fast")
    for key in keys:
        assert np.array_equal(got[key], ref[key]), key
    assert ref["ssf_steps"].sum() > 0
    H = _spacetime(2)
    syn, rd = oracle_lib.sample_storage(HZ, 2, 0.01, 0.01, seed=8, stream=1, shot0=0, B=600)
    lz = code225.logicals.z
    dec = Decoder(H, 0.0067, method="ms", precision="f32", max_iter=30, n_data=225, fold_blocks=3, logicals=lz)
    got = dec.decode(syn, readout=rd, want=("corr", "iters", "status", "fail"))
    ref = oracle_lib.decode(H, 0.0067, syn, method="ms", precision="f32", max_iter=30, n_data=225, fold_blocks=3,
                            lz=lz, readout=rd, want_llr=False)
    for key in ("corr", "iters", "status", "fail"):
        assert np.array_equal(got[key], ref[key]), key


@pytest.fixture(params=["compact", "onepass"])
def lean_path(request, monkeypatch):
    """Lean launches run the two-pass compact path (ms_triage_kernel +
    bp_ms_cmp_kernel) by default; QD_OPT_COMPACT = 0 keeps the one-pass
    bp_ms_wave_kernel.  Lean tests run both."""
    from exp_ldpc_amd import decoder
    if request.param == "onepass":
        monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "compact", 0)
    return request.param


@pytest.fixture(params=["fused", "queue"])
def ssf_path(request, monkeypatch):
    """Two-pass SSF decodes queue BP-failed shots for ssf_lut_kernel by default
    (QD_OPT_SSF_FUSE = 0); 1 runs SSF inside the compact BP kernel."""
    from exp_ldpc_amd import decoder
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "ssf_fuse", 1 if request.param == "fused" else 0)
    return request.param


@pytest.mark.parametrize("precision,occupancy", [("f64", 0), ("f64", 12), ("f32", 0)])
def test_bench_lean_kernels_all_points(gpu_available, oracle_lib, precision, occupancy, lean_path, ssf_path):
    """The benchmarked instantiation (bp_ms_wave_kernel<.., LEAN=true, ..>, chosen
    when x / corr / llr are all null) pinned bit-exactly: exactly bench.py's
    decode_device call (syn + readout in; iters, status, ssf_steps, fail out) at
    all 9 sweep points, 4096 device-sampled shots each (bench.py's sampler
    streams, shot offset of its step 3), f64 headline and f32 variant, every
    output compared with the oracle on the same shots.  f64 also at 12 waves per
    CU (bench.py's overlapped phases: the 3-waves-per-SIMD build)."""
    import torch
    from exp_ldpc_amd.decoder import Decoder
    code = load_code("hgp_12_3_4_s1234")
    hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
    dev = torch.device("cuda", 0)
    B, seed, shot0 = 4096, 20250221, 3 * (1 << 18)
    for pi, p in enumerate(np.geomspace(1e-3, 1e-1, 9)):
        dec = Decoder(hz, 2 * p / 3, method="ms", precision=precision, max_iter=50, ms_scaling=0.0,
                      flip_sets=hx, logicals=lz)
        if occupancy:
            dec.set_wave_occupancy(occupancy)
        syn = torch.empty((B, hz.shape[0]), dtype=torch.uint8, device=dev)
        rd = torch.empty((B, hz.shape[1]), dtype=torch.uint8, device=dev)
        dec.sample_storage_device(0, p, p, seed, pi, shot0, B, syn, rd)
        out = {k: torch.empty(B, dtype=dt, device=dev) for k, dt in
               (("iters", torch.int32), ("status", torch.uint8), ("ssf_steps", torch.int32), ("fail", torch.uint8))}
        dec.decode_device(B, syn=syn, readout=rd, **out)
        torch.cuda.synchronize()
        bp_k, ssf_k, pre_k = dec.last_kernels()
        assert ("cmp_kernel" in bp_k and "triage" in pre_k) == (lean_path == "compact"), (bp_k, pre_k)
        # fused: no SSF launch, the compact kernel's FUSE argument is the generators per lane
        fused = lean_path == "compact" and ssf_path == "fused"
        assert (ssf_k == "") == fused and (bp_k.endswith(", 2>") if fused else True), (bp_k, ssf_k)
        rs, rr = oracle_lib.sample_storage(hz, 0, p, p, seed=seed, stream=pi, shot0=shot0, B=B)
        assert np.array_equal(syn.cpu().numpy(), rs) and np.array_equal(rd.cpu().numpy(), rr), p
        ref = oracle_lib.decode(hz, 2 * p / 3, rs, method="ms", precision=precision, max_iter=50, ssf=True, gens=hx,
                                lz=lz, readout=rr, want_llr=False, ssf_impl="fast")
        for k in out:
            assert np.array_equal(out[k].cpu().numpy(), ref[k]), (p, k)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_lean_zero_syndrome_shortcut_and_nonpositive_priors(gpu_available, oracle_lib, precision, lean_path):
    """The LEAN kernel writes iteration 1 / converged / x = 0 directly for an
    all-zero syndrome only when every prior LLR is > 0.  Per-column priors with
    some p >= 0.5 (LLR <= 0: BP must run and need not converge at once) and the
    same shots with all p < 0.5, a quarter of them zero syndromes: iterations,
    status, SSF steps and failure flags equal the oracle's in both cases."""
    import torch
    from exp_ldpc_amd.decoder import Decoder
    code = load_code("hgp_12_3_4_s1234")
    hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
    rng = np.random.default_rng(11)
    B, n = 2048, hz.shape[1]
    e = (rng.random((B, n)) < 0.01).astype(np.uint8)
    e[: B // 4] = 0
    syn = np.ascontiguousarray(((hz @ e.T).T % 2).astype(np.uint8))
    rd = (e ^ (rng.random((B, n)) < 0.002)).astype(np.uint8)
    dev = torch.device("cuda", 0)
    for probs in (rng.uniform(0.005, 0.02, n), np.where(np.arange(n) % 37 == 0, 0.6, 0.01)):
        dec = Decoder(hz, probs, method="ms", precision=precision, max_iter=30, flip_sets=hx, logicals=lz)
        out = {k: torch.empty(B, dtype=dt, device=dev) for k, dt in
               (("iters", torch.int32), ("status", torch.uint8), ("ssf_steps", torch.int32), ("fail", torch.uint8))}
        dec.decode_device(B, syn=torch.from_numpy(syn).to(dev), readout=torch.from_numpy(rd).to(dev), **out)
        torch.cuda.synchronize()
        ref = oracle_lib.decode(hz, probs, syn, method="ms", precision=precision, max_iter=30, ssf=True, gens=hx,
                                lz=lz, readout=rd, want_llr=False, ssf_impl="fast")
        for k in out:
            assert np.array_equal(out[k].cpu().numpy(), ref[k]), (probs.max(), k)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_wave_occupancy_does_not_change_results(gpu_available, oracle_lib, precision, lean_path):
    """qd_graph_set_wave_occupancy (bench.py's overlapped phases use 12 f64
    waves per CU) only changes the persistent grid: iterations, status, SSF
    steps and failure flags equal the oracle's at 4, 12 and the default; an
    out-of-range value is refused."""
    import torch
    from exp_ldpc_amd._abi import QdecError
    from exp_ldpc_amd.decoder import Decoder
    code = load_code("hgp_12_3_4_s1234")
    hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
    p, B = 0.05, 6000
    dec = Decoder(hz, 2 * p / 3, method="ms", precision=precision, max_iter=50, flip_sets=hx, logicals=lz)
    dev = torch.device("cuda", 0)
    syn = torch.empty((B, hz.shape[0]), dtype=torch.uint8, device=dev)
    rd = torch.empty((B, hz.shape[1]), dtype=torch.uint8, device=dev)
    dec.sample_storage_device(0, p, p, 7, 0, 0, B, syn, rd)
    rs, rr = syn.cpu().numpy(), rd.cpu().numpy()
    ref = oracle_lib.decode(hz, 2 * p / 3, rs, method="ms", precision=precision, max_iter=50, ssf=True, gens=hx,
                            lz=lz, readout=rr, want_llr=False, ssf_impl="fast")
    for w in (4, 12, 0):
        dec.set_wave_occupancy(w)
        out = {k: torch.empty(B, dtype=dt, device=dev) for k, dt in
               (("iters", torch.int32), ("status", torch.uint8), ("ssf_steps", torch.int32), ("fail", torch.uint8))}
        dec.decode_device(B, syn=syn, readout=rd, **out)
        torch.cuda.synchronize()
        for k in out:
            assert np.array_equal(out[k].cpu().numpy(), ref[k]), (w, k)
    with pytest.raises(QdecError):
        dec.set_wave_occupancy(-1)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_lean_zero_messages(gpu_available, oracle_lib, precision, lean_path):
    """Exact zero messages on the LEAN kernel.  The f64 LEAN kernel reads ldpc's
    sign test `v <= 0` from sign bits (QDEC_MS_SIGNBIT) and takes a rare path for
    check rows holding a zero entry (+0 or -0).  Priors of exactly 0 (p = 0.5:
    log(1) = +0) put +0 messages into the rows from iteration 1; a mix of p = 0.5
    and p = 0.5 +- tiny steps gives +0, -0-producing sums and sign changes, and all
    columns at 0.5 makes every row all-zero.  Iterations, status, SSF steps and
    failure flags equal the oracle's (compare-based) in every case."""
    import torch
    from exp_ldpc_amd.decoder import Decoder
    code = load_code("hgp_12_3_4_s1234")
    hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
    rng = np.random.default_rng(5)
    B, n = 3000, hz.shape[1]
    e = (rng.random((B, n)) < 0.03).astype(np.uint8)
    syn = np.ascontiguousarray(((hz @ e.T).T % 2).astype(np.uint8))
    rd = (e ^ (rng.random((B, n)) < 0.01)).astype(np.uint8)
    dev = torch.device("cuda", 0)
    cases = (np.where(np.arange(n) % 5 == 0, 0.5, 0.02),
             np.where(np.arange(n) % 3 == 0, 0.5, np.where(np.arange(n) % 3 == 1, 0.3, 0.7)),
             np.full(n, 0.5))
    for ci, probs in enumerate(cases):
        dec = Decoder(hz, probs, method="ms", precision=precision, max_iter=25, flip_sets=hx, logicals=lz)
        out = {k: torch.empty(B, dtype=dt, device=dev) for k, dt in
               (("iters", torch.int32), ("status", torch.uint8), ("ssf_steps", torch.int32), ("fail", torch.uint8))}
        dec.decode_device(B, syn=torch.from_numpy(syn).to(dev), readout=torch.from_numpy(rd).to(dev), **out)
        torch.cuda.synchronize()
        ref = oracle_lib.decode(hz, probs, syn, method="ms", precision=precision, max_iter=25, ssf=True, gens=hx,
                                lz=lz, readout=rd, want_llr=False, ssf_impl="fast")
        for k in out:
            assert np.array_equal(out[k].cpu().numpy(), ref[k]), (ci, k)
