"""CPU-side checks of the product library and host logic: the C ABI loads and
exports every symbol include/qdec.h declares, constructors fail loudly without
a GPU, OSD (host C++ in libqdec_hip.so) matches its independent checker, and the
harness argument handling mirrors the reference."""
import argparse

import numpy as np
import scipy.sparse as sp
import pytest

from conftest import load_checks

HX, HZ = load_checks("hgp_12_3_4_s1234")


def test_library_exports_every_header_symbol():
    from exp_ldpc_amd import _abi
    lib = _abi.load()
    syms = _abi.header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _abi.SIGNATURES, f"{s} has no ctypes signature"
    assert lib.qd_abi_version() == 1


def test_no_cpu_fallback_without_gpu():
    """On a machine without a HIP device the decoder refuses to construct."""
    from exp_ldpc_amd import _abi
    from exp_ldpc_amd.decoder import Decoder
    if _abi.load().qd_device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(_abi.QdecError):
        Decoder(HZ, 0.01)


def test_missing_library_fails_loudly(tmp_path):
    from exp_ldpc_amd import _abi
    with pytest.raises(_abi.QdecError):
        _abi.load(str(tmp_path / "nope.so"))


@pytest.mark.parametrize("method,order", [("osd0", 0), ("osd_cs", 7), ("osd_cs", 3), ("osd_e", 4)])
def test_osd_matches_checker(method, order):
    from exp_ldpc_amd.osd import OsdSolver
    from oracle.osd_py import osd_decode
    rng = np.random.default_rng(order)
    B = 20
    e = (rng.random((B, 225)) < 0.05).astype(np.uint8)
    syn = ((HZ @ e.T).T % 2).astype(np.uint8)
    llr = rng.normal(3, 3, (B, 225))
    llr[:, :10] = 1.0  # ties: order by column index
    o0, ow = OsdSolver(HZ, method, order).solve(syn, llr)
    for b in range(B):
        r0, rw = osd_decode(HZ, syn[b], llr[b], method, order)
        assert np.array_equal(o0[b], r0) and np.array_equal(ow[b], rw)
        assert ((HZ @ ow[b]) % 2 == syn[b]).all()
        assert ow[b].sum() <= o0[b].sum()


def test_osd_on_spacetime_matrix():
    from exp_ldpc_amd.osd import OsdSolver
    from exp_ldpc_amd.spacetime import SpacetimeCode
    from oracle.osd_py import osd_decode
    H = SpacetimeCode(HZ, 1).spacetime_check_matrix
    rng = np.random.default_rng(9)
    e = (rng.random((6, H.shape[1])) < 0.03).astype(np.uint8)
    syn = ((H @ e.T).T % 2).astype(np.uint8)
    llr = rng.normal(2, 2, (6, H.shape[1]))
    o0, ow = OsdSolver(H, "osd_cs", 7).solve(syn, llr)
    for b in range(6):
        r0, rw = osd_decode(H, syn[b], llr[b], "osd_cs", 7)
        assert np.array_equal(ow[b], rw)


def test_bp_method_names():
    from exp_ldpc_amd import _abi
    from exp_ldpc_amd.decoder import parse_bp_method
    for name in ("ps", "product_sum", 0, "0"):
        assert parse_bp_method(name) == _abi.QD_PRODUCT_SUM
    for name in ("ms", "msl", "minimum_sum", "minimum_sum_log", "min_sum", 1, 3):
        assert parse_bp_method(name) == _abi.QD_MIN_SUM
    with pytest.raises(NotImplementedError):
        parse_bp_method("ps_log")
    with pytest.raises(ValueError):
        parse_bp_method("bogus")


def test_ldpc_kwargs_resolution():
    from exp_ldpc_amd.ldpc_compat import _resolve_probs
    assert np.allclose(_resolve_probs(4, {"error_rate": 0.1}), 0.1)
    assert np.allclose(_resolve_probs(3, {"channel_probs": [0.1, 0.2, 0.3]}), [0.1, 0.2, 0.3])
    assert np.allclose(_resolve_probs(2, {"channel_prior": [0.1, 0.2]}), [0.1, 0.2])  # _experiment.py:77
    assert np.allclose(_resolve_probs(2, {"channel_probs": [None], "error_rate": 0.3}), 0.3)
    with pytest.raises(ValueError):
        _resolve_probs(3, {})
    with pytest.raises(ValueError):
        _resolve_probs(3, {"channel_probs": [0.1, 0.2]})


def test_harness_arguments_mirror_reference():
    from exp_ldpc_amd.codes import QuantumCode, QuantumCodeChecks
    from exp_ldpc_amd.experiment import add_bposd_args, parse_sweep_spec, unpack_bposd_args
    p = argparse.ArgumentParser()
    add_bposd_args(p)
    a = p.parse_args([])
    code = QuantumCode(QuantumCodeChecks(HX, HZ))
    opts = unpack_bposd_args(a, code)
    assert opts == {"max_iter": 225, "bp_method": "ps", "ms_scaling_factor": 0, "osd_method": "osd_cs",
                    "osd_order": 7}
    assert parse_sweep_spec("(1e-3, 1e-1, 9)") == (1e-3, 1e-1, 9)
    with pytest.raises(RuntimeError):
        parse_sweep_spec("(0.2, 0.1, 3)")
    with pytest.raises(RuntimeError):
        parse_sweep_spec("0.1,0.2")


def test_qldpc_shim_surface():
    import qldpc
    import qldpc.misc
    assert callable(qldpc.misc.p_sweep_main)
    nm = qldpc.noise_model.depolarizing_noise(0.01, 0.01)
    assert nm.kind == "depolarizing"
    assert qldpc.read_quantum_code is not None and qldpc.SpacetimeCode is not None


def test_sharding_arithmetic():
    from exp_ldpc_amd.sharding import shard_range, step_shot0
    assert [shard_range(10, 3, r) for r in range(3)] == [(0, 4), (4, 8), (8, 10)]
    seen = set()
    for s in range(3):
        for r in range(4):
            lo = step_shot0(s, 4, r, 5)
            seen.update(range(lo, lo + 5))
    assert seen == set(range(60))


def test_checkpoint_fingerprint_covers_noise_configuration():
    """A restarted sweep must not reuse a row computed under another noise model
    argument (pm), prior function or noise model."""
    from exp_ldpc_amd.codes import QuantumCode, QuantumCodeChecks
    from exp_ldpc_amd.experiment import _config_fingerprint
    from exp_ldpc_amd.noise_model import depolarizing_noise, circuit_noise
    hx, hz = load_checks("hgp_12_3_4_s1234")
    code = QuantumCode(QuantumCodeChecks(hx, hz))
    opts = {"max_iter": 30, "bp_method": "ms"}
    base = (code, 0, "bpssf", opts, "f64", 5, 4000, 0)
    p = 0.01
    fp = lambda model, args, dp, mp: _config_fingerprint(*base, noise=(model, args, dp, mp))
    ref = fp(depolarizing_noise, dict(p=p, pm=p), 2 * p / 3, 2 * p / 3)
    assert ref == fp(depolarizing_noise, dict(pm=p, p=p), 2 * p / 3, 2 * p / 3)  # order-free
    assert ref != fp(depolarizing_noise, dict(p=p, pm=2 * p), 2 * p / 3, 2 * p / 3)
    assert ref != fp(depolarizing_noise, dict(p=p, pm=p), p, 2 * p / 3)
    assert ref != fp(depolarizing_noise, dict(p=p, pm=p), 2 * p / 3, p)
    assert ref != fp(circuit_noise, dict(p=p, pm=p), 2 * p / 3, 2 * p / 3)
    assert ref != _config_fingerprint(*base)  # rows fingerprinted without noise are not reused either


def test_checkpoint_append_keeps_file_parseable(tmp_path):
    """Rows with a different column set (older format, other decoder options)
    are merged under a union header, so the next restart can read the CSV."""
    import pandas as pd
    from exp_ldpc_amd.experiment import _append_checkpoint_row, _load_checkpoint
    ck = str(tmp_path / "sweep.csv")
    pd.DataFrame.from_records([{"p_ph": 0.01, "failures": 3, "samples": 100}]).to_csv(ck, index=False)  # old format
    _append_checkpoint_row(ck, {"p_ph": 0.02, "failures": 5, "samples": 100, "precision": "f64", "config_fp": "ab"})
    _append_checkpoint_row(ck, {"p_ph": 0.03, "failures": 7, "samples": 100, "precision": "f64", "config_fp": "cd"})
    _append_checkpoint_row(ck, {"p_ph": 0.04, "failures": 9, "samples": 100, "precision": "f64", "config_fp": "ef",
                                "osd_order": 7})
    df = pd.read_csv(ck, float_precision="round_trip")
    assert list(df["p_ph"]) == [0.01, 0.02, 0.03, 0.04] and list(df["failures"]) == [3, 5, 7, 9]
    assert "osd_order" in df.columns and df["osd_order"].isna().sum() == 3
    rows = _load_checkpoint(ck)
    assert set(rows) == {(0.02, "ab"), (0.03, "cd"), (0.04, "ef")}
    with open(ck, "a") as f:  # a corrupt tail: loading reuses nothing, the next append sets the file aside
        f.write("1,2,3,4,5,6,7,8,9,10,11\n")
    assert _load_checkpoint(ck) == {}
    _append_checkpoint_row(ck, {"p_ph": 0.05, "failures": 1, "samples": 100, "precision": "f64", "config_fp": "gh"})
    assert set(_load_checkpoint(ck)) == {(0.05, "gh")}


def test_sparse_logicals_accepted_and_copied():
    """QuantumCodeLogicals keeps scipy-sparse logicals as a private CSR copy
    (config 5's k = 4080 never goes dense); dense inputs stay read-only."""
    from exp_ldpc_amd.codes import QuantumCodeLogicals
    lz = sp.random(6, 40, density=0.1, format="coo", random_state=1, dtype=np.float64)
    lz.data[:] = 1
    lz = lz.astype(np.uint8)
    q = QuantumCodeLogicals(lz.tocsc(), lz)
    assert sp.isspmatrix_csr(q.x) and q.num_logicals == 6 and q.num_qubits == 40
    assert np.array_equal(q.z.toarray(), lz.toarray())
    q.z.data[:] = 0                     # the caller's matrix is untouched
    assert lz.toarray().any()
    with pytest.raises(TypeError):
        QuantumCodeLogicals(lz.astype(np.float32), lz)
    d = QuantumCodeLogicals(lz.toarray(), lz.toarray())
    assert not d.x.flags.writeable


def test_run_shards_retries_a_failed_shard_once_in_a_fresh_thread():
    """p_sweep's fan-out (reference misc/p_sweep.py:24-40): a shard that raises
    is re-run once in a new worker thread on the same device; counters are
    summed over shards exactly once."""
    import threading

    from exp_ldpc_amd.experiment import run_shards
    calls = []

    def work(d, lo, hi, attempt):
        calls.append((d, lo, hi, attempt, threading.current_thread().name))
        if d == 1 and attempt == 0:
            raise RuntimeError("injected shard failure")
        return [hi - lo, 1, 0.5]

    out = run_shards([(0, 0, 10), (1, 10, 25), (2, 25, 30)], work, p_ph=0.01)
    assert out == [30, 3, 1.5]
    first = [c for c in calls if c[3] == 0]
    retry = [c for c in calls if c[3] == 1]
    assert len(first) == 3 and [c[:3] for c in retry] == [(1, 10, 25)]
    assert retry[0][4] != next(c[4] for c in first if c[0] == 1)  # a fresh worker thread


def test_run_shards_reports_the_failed_range():
    from exp_ldpc_amd.experiment import ShardError, run_shards

    def work(d, lo, hi, attempt):
        if lo == 10:
            raise ValueError("broken device")
        return [1]

    with pytest.raises(ShardError) as ei:
        run_shards([(0, 0, 10), (0, 10, 20)], work, p_ph=0.02)
    e = ei.value
    assert (e.p_ph, e.device, e.lo, e.hi) == (0.02, 0, 10, 20) and "shots [10, 20)" in str(e)
    # one device: the first attempt runs inline, the retry in a thread
    seen = []

    def once(d, lo, hi, attempt):
        seen.append(attempt)
        if attempt == 0:
            raise RuntimeError("transient")
        return [hi - lo]

    assert run_shards([(0, 0, 7)], once) == [7] and seen == [0, 1]


def test_run_shards_does_not_retry_device_errors():
    """A HIP error (library status <= -100, or torch's HIP RuntimeError) is
    sticky on its device: no retry, ShardError at once naming that shard."""
    from exp_ldpc_amd._abi import QdecError
    from exp_ldpc_amd.experiment import ShardError, device_error, run_shards
    assert device_error(QdecError("decode launch failed", -101)) and not device_error(QdecError("bad arg", -7))
    assert device_error(RuntimeError("HIP error: an illegal memory access")) and not device_error(ValueError("x"))
    for exc in (QdecError("qd_decode_batch_device failed (-101)", -101), RuntimeError("HIP error: launch failure")):
        seen = []

        def work(d, lo, hi, attempt, exc=exc):
            seen.append((lo, attempt))
            if lo == 5:
                raise exc
            return [1]

        with pytest.raises(ShardError) as ei:
            run_shards([(0, 0, 5), (1, 5, 9)], work, p_ph=0.03)
        assert (ei.value.device, ei.value.lo) == (1, 5) and all(a == 0 for _, a in seen)


def test_set_logicals_rejects_1d_dense_input():
    """A 1-D dense logicals argument is malformed (k x n_data expected); it must
    not be read as a single logical row.  Checked before any device call."""
    from exp_ldpc_amd.decoder import Decoder
    d = Decoder.__new__(Decoder)
    d.n_data = 5
    with pytest.raises(ValueError, match="k x n_data"):
        Decoder.set_logicals(d, np.ones(5, np.uint8))


def _host_graph(lib, H, n_data=None, gens=None, lz=None, probs=None):
    import ctypes as C

    from exp_ldpc_amd import _abi
    H = sp.csr_matrix(H)
    H.sort_indices()
    rp = np.ascontiguousarray(H.indptr, np.int32)
    ci = np.ascontiguousarray(H.indices, np.int32)
    h = C.c_void_p()
    nd = n_data or H.shape[1]
    _abi.check(lib.qd_graph_create_host(H.shape[0], H.shape[1], _abi.ptr(rp), _abi.ptr(ci), nd, 1, C.byref(h)),
               "qd_graph_create_host")
    if gens is not None:
        G = sp.csr_matrix(gens)
        G.sort_indices()
        gp, gi = np.ascontiguousarray(G.indptr, np.int32), np.ascontiguousarray(G.indices, np.int32)
        _abi.check(lib.qd_graph_set_flipsets(h, G.shape[0], _abi.ptr(gp), _abi.ptr(gi)), "flipsets")
    if lz is not None:
        L = sp.csr_matrix(lz)
        L.sort_indices()
        lp, li = np.ascontiguousarray(L.indptr, np.int32), np.ascontiguousarray(L.indices, np.int32)
        _abi.check(lib.qd_graph_set_logicals_csr(h, L.shape[0], _abi.ptr(lp), _abi.ptr(li)), "logicals")
    if probs is not None:
        pr = np.ascontiguousarray(np.broadcast_to(np.asarray(probs, np.float64), (H.shape[1],)))
        _abi.check(lib.qd_graph_set_priors(h, _abi.ptr(pr)), "priors")
    d, nb = C.c_uint64(0), C.c_int64(0)
    _abi.check(lib.qd_graph_table_digest(h, C.byref(d), C.byref(nb)), "digest")
    return h, d.value, nb.value


def test_host_only_tables_build_without_a_gpu(code225):
    """qd_graph_create_host runs the host half of graph setup -- validation,
    wave-kernel layout anneals (ms_layout), flip-set inverse tables, logicals,
    priors -- with no device: deterministic tables, and decodes refuse the
    handle.  tools/sanitize.sh runs this under ASan + UBSan."""
    import ctypes as C

    from exp_ldpc_amd import _abi
    lib = _abi.load()
    hz, hx, lz = code225.checks.z, code225.checks.x, code225.logicals.z
    h1, d1, b1 = _host_graph(lib, hz, gens=hx, lz=lz, probs=0.01)
    h2, d2, b2 = _host_graph(lib, hz, gens=hx, lz=lz, probs=0.01)
    assert d1 == d2 and b1 == b2 and b1 > 10_000
    h3, d3, _ = _host_graph(lib, hz, gens=hx, lz=lz, probs=0.02)  # other priors: other tables
    assert d3 != d1
    prm = _abi.QdParams(50, _abi.QD_MIN_SUM, _abi.QD_F64, 0, 0, 0, 0.0)
    syn = np.zeros((1, hz.shape[0]), np.uint8)
    rc = lib.qd_decode_batch(h1, C.byref(prm), 1, _abi.ptr(syn), None, None, None, None, None, None, None, None,
                             None)
    assert rc != 0 and b"host-only" in lib.qd_last_error()
    # ragged random graphs (workgroup-kernel shapes and degree-0 rows/columns)
    rng = np.random.default_rng(5)
    for m, n in ((30, 50), (300, 700), (700, 1500)):
        A = sp.random(m, n, density=4.0 / n, random_state=rng, format="csr")
        A.data[:] = 1
        h, d, b = _host_graph(lib, A, probs=rng.uniform(0.001, 0.2, n))
        assert b > 0
        lib.qd_graph_destroy(h)
    for h in (h1, h2, h3):
        assert lib.qd_graph_destroy(h) == 0


def _lut_ssf_emulate(tab, H, gens, x, resid, max_steps=0):
    """The table-driven SSF kernel's steps (ssf_lut_kernel, qdec_bp.hip) run on
    the host over the library's own tables: local syndromes from the toggle rows
    of the violated checks, then per step the table entry of every generator,
    the max of (rank, -g), the winner's subset applied (qubits x, toggle rows of
    the checks it flips).  Returns (x, steps)."""
    lut, off, lcw, tog, gp = tab
    x = x.copy()
    ng = gens.shape[0]
    gq = [gens.indices[gens.indptr[g]:gens.indptr[g + 1]] for g in range(ng)]
    sl = np.zeros(ng, np.int64)
    for c in np.flatnonzero(resid):
        for g in range(ng):
            sl[g] ^= (int(tog[c, g & 63]) >> (16 * (g >> 6))) & 0xffff
    sw = int(resid.sum())
    steps = 0
    while sw > 0 and (max_steps <= 0 or steps < max_steps):
        best, bg = 0, -1
        for g in range(ng):
            e = int(lut[off[g] + sl[g]])
            if e >> 24:
                key = ((e >> 24) << 15) | ((127 - g) << 8) | (e & 0xff)
                if key > best:
                    best, bg = key, g
        if bg < 0:
            break
        e = int(lut[off[bg] + sl[bg]])
        t, fm = e & 0xff, (e >> 8) & 0xffff
        slg = int(sl[bg])
        sw -= bin(slg).count("1") - bin(slg ^ fm).count("1")
        steps += 1
        for b in range(16):
            if (fm >> b) & 1:
                c = (int(lcw[b // 4, bg]) >> (8 * (b % 4))) & 0xff
                for g in range(ng):
                    sl[g] ^= (int(tog[c, g & 63]) >> (16 * (g >> 6))) & 0xffff
        for k in range(len(gq[bg])):
            if (t >> k) & 1:
                x[gq[bg][k]] ^= 1
    return x, steps


def _lut_tables(lib, h):
    import ctypes as C

    from exp_ldpc_amd import _abi
    has, nb = C.c_int32(0), C.c_int64(0)
    _abi.check(lib.qd_graph_ssf_tables(h, C.byref(has), C.byref(nb)), "ssf_tables")
    if not has.value:
        return None
    gp, mp = C.c_int32(0), C.c_int32(0)
    _abi.check(lib.qd_graph_ssf_tables_copy(h, None, None, None, None, C.byref(gp), C.byref(mp)), "copy")
    lut = np.zeros(nb.value // 4, np.uint32)
    off = np.zeros(gp.value, np.uint32)
    lcw = np.zeros((4, gp.value), np.uint32)
    tog = np.zeros((mp.value + 1, 64), np.uint32)
    _abi.check(lib.qd_graph_ssf_tables_copy(h, _abi.ptr(lut), _abi.ptr(off), _abi.ptr(lcw), _abi.ptr(tog), None,
                                            None), "copy")
    return lut, off, lcw, tog, gp.value


@pytest.mark.parametrize("max_steps", [0, 2])
def test_ssf_lut_tables_follow_the_spec(code225, oracle_lib, max_steps):
    """The table-driven SSF kernel's tables (ssf_lut_tables, qdec_abi.cpp) on the
    n = 225 HGP code: every generator shares ONE 4096-entry score table (same
    4 x 3 local pattern after the canonical local-check order), and the kernel's
    step rule run on the host over those exact tables reproduces the oracle's
    SSF (oracle/qdec_oracle.c ssf_run_fast: x and step counts) on BP-failed
    shots."""
    from exp_ldpc_amd import _abi
    lib = _abi.load()
    hz, hx, lz = code225.checks.z, code225.checks.x, code225.logicals.z
    h, _, _ = _host_graph(lib, hz, gens=hx, lz=lz, probs=0.02)
    try:
        tab = _lut_tables(lib, h)
        assert tab is not None
        lut, off = tab[0], tab[1]
        assert lut.size == 4096 and not off[:hx.shape[0]].any()
        assert not tab[3][-1].any()  # the zero toggle row the kernel reads for unflipped bits
        ranks = sorted({int(e) >> 24 for e in lut} - {0})
        assert ranks == list(range(1, len(ranks) + 1))
        rng = np.random.default_rng(11)
        B = 160
        err = (rng.random((B, hz.shape[1])) < 0.06).astype(np.uint8)
        syn = ((hz @ err.T).T % 2).astype(np.uint8)
        hx = sp.csr_matrix(hx)
        hx.sort_indices()
        bp = oracle_lib.decode(hz, 0.02, syn, method="ms", precision="f64", max_iter=1, ssf=False, want_llr=False)
        ref = oracle_lib.decode(hz, 0.02, syn, method="ms", precision="f64", max_iter=1, ssf=True, gens=hx,
                                ssf_max_steps=max_steps, want_llr=False)
        checked = 0
        for b in np.flatnonzero((bp["status"] & 1) == 0):
            resid = (syn[b] ^ (hz @ bp["x"][b]) % 2).astype(np.uint8)
            x, steps = _lut_ssf_emulate(tab, hz, hx, bp["x"][b], resid, max_steps)
            assert np.array_equal(x, ref["x"][b]) and steps == ref["ssf_steps"][b], b
            checked += 1
        assert checked > 100 and ref["ssf_steps"].sum() > 200
    finally:
        lib.qd_graph_destroy(h)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_host_only_it1_tables_equal_the_oracle_iteration_1(code225, oracle_lib, precision):
    """The triage's iteration-1 tables (it1_tables, qdec_abi.cpp), built by a
    host-only graph: for random per-column priors (with exact ties) and random
    syndromes, looking up each column's decision under its checks' syndrome
    pattern equals the oracle's hard decision after min-sum iteration 1
    (ldpc v1 restatement, max_iter = 1).  A non-positive prior builds no
    table for the precision.  tools/sanitize.sh runs this under ASan + UBSan."""
    import ctypes as C

    from exp_ldpc_amd import _abi
    lib = _abi.load()
    hz = sp.csr_matrix(code225.checks.z)
    m, n = hz.shape
    rng = np.random.default_rng(3)
    probs = rng.choice([0.001, 0.01, 0.02, 0.05, 0.1], size=n)  # ties inside rows
    h, _, _ = _host_graph(lib, hz, probs=probs)
    try:
        prec = _abi.QD_F64 if precision == "f64" else _abi.QD_F32
        npad = C.c_int32(0)
        _abi.check(lib.qd_graph_it1_tables_copy(h, prec, None, None, C.byref(npad)), "it1 copy")
        lut = np.zeros(npad.value, np.uint16)
        vchk = np.zeros(npad.value, np.uint64)
        _abi.check(lib.qd_graph_it1_tables_copy(h, prec, _abi.ptr(lut), _abi.ptr(vchk), None), "it1 copy")
        B = 400
        syn = (rng.random((B, m)) < 0.08).astype(np.uint8)
        ref = oracle_lib.decode(hz, probs, syn, method="ms", precision=precision, max_iter=1, want_llr=False)
        synp = np.concatenate([syn, np.zeros((B, 1), np.uint8)], axis=1)  # pad check id m -> 0
        ids = np.stack([((vchk[:n] >> np.uint64(16 * k)) & np.uint64(0xffff)).astype(np.int64) for k in range(4)], 1)
        pat = sum(synp[:, ids[:, k]].astype(np.int64) << k for k in range(4))
        got = ((lut[:n].astype(np.int64)[None, :] >> pat) & 1).astype(np.uint8)
        assert np.array_equal(got, ref["x"])
    finally:
        lib.qd_graph_destroy(h)
    h2, _, _ = _host_graph(lib, hz, probs=np.where(np.arange(n) == 7, 0.6, 0.01))  # a negative LLR
    try:
        assert lib.qd_graph_it1_tables_copy(h2, _abi.QD_F64, None, None, None) != 0
    finally:
        lib.qd_graph_destroy(h2)


def test_host_only_queue_layout(code225):
    """The queue scratch layout attach_queue allocates (queue_layout,
    qdec_abi.cpp), computed on a host-only graph for batches around the
    64-shot tile and segment sizes: regions in order and disjoint, the compact
    list's counters on a 256-B boundary (u64 atomics) and its entry region
    16-B aligned, and enough segment capacity for every
    shot of every tile (tile t -> segment t mod 64)."""
    from exp_ldpc_amd import _abi
    lib = _abi.load()
    hz = code225.checks.z
    h, _, _ = _host_graph(lib, hz, gens=code225.checks.x, probs=0.01)
    try:
        m, n = hz.shape
        for B in (1, 63, 64, 65, 4095, 4097, 64 * 64 + 1, 1 << 18, (1 << 18) + 13):
            out = np.zeros(8, np.int64)
            _abi.check(lib.qd_graph_queue_layout(h, B, _abi.ptr(out)), "layout")
            total, idx, x, r, cnt, cmp, cap, ent = (int(v) for v in out)
            assert idx == 256 and x == idx + 8 * B and r == x + B * n
            packed = 8 * (1 + 2 * 256 // 64 + 128 // 64)
            assert cnt >= x + B * max(n + m, packed) and cnt % 256 == 0
            # two lists (light, heavy) of 64 segments, every segment able to
            # hold all of its tiles' shots
            assert cmp == cnt + 2 * 64 * 128 and cmp % 16 == 0 and ent == 8 * (1 + 2 + 4)
            tiles = -(-B // 64)
            assert cap * 64 >= B and cap >= 64 * (-(-tiles // 64)) and cap % 64 == 0
            assert total >= cmp + 2 * 64 * cap * ent
    finally:
        lib.qd_graph_destroy(h)


def test_kernel_options_are_handle_state_not_environment(code225):
    """Kernel choices are per-handle options (qd_graph_set_option): defaults,
    round trip, range checks, unknown options refused; and no source file of
    the library reads the environment (every knob of earlier rounds that
    switched a kernel per launch by getenv is gone or an option)."""
    import ctypes as C
    import glob
    import os
    import re

    from exp_ldpc_amd import _abi
    from exp_ldpc_amd.decoder import OPTIONS
    from conftest import REPO
    lib = _abi.load()
    h, _, _ = _host_graph(lib, code225.checks.z, gens=code225.checks.x, probs=0.01)
    try:
        v = C.c_int32(0)
        defaults = {"compact": 1, "triage_it1": 1, "ssf": 0, "lds_kernel": -1, "group_kernel": -1, "ssf_inc": 1,
                    "block_wg": 0, "group_mb": 0}
        for name, d in defaults.items():
            _abi.check(lib.qd_graph_get_option(h, OPTIONS[name], C.byref(v)), name)
            assert v.value == d, name
        for name, val in (("compact", 0), ("ssf", 3), ("lds_kernel", 1), ("group_mb", 512)):
            _abi.check(lib.qd_graph_set_option(h, OPTIONS[name], val), name)
            _abi.check(lib.qd_graph_get_option(h, OPTIONS[name], C.byref(v)), name)
            assert v.value == val
        assert lib.qd_graph_set_option(h, OPTIONS["ssf"], 4) == -2
        assert lib.qd_graph_set_option(h, OPTIONS["compact"], 2) == -2
        assert lib.qd_graph_set_option(h, 99, 0) == -2
        has, nb = C.c_int32(0), C.c_int64(0)
        _abi.check(lib.qd_graph_ssf_tables(h, C.byref(has), C.byref(nb)), "tables")
        assert has.value == 1 and nb.value == 4096 * 4
    finally:
        lib.qd_graph_destroy(h)
    srcs = glob.glob(os.path.join(REPO, "exp_ldpc_amd", "csrc", "*"))
    assert srcs
    for f in srcs:
        assert not re.search(r"\bgetenv\s*\(", open(f).read()), f


def test_hgp_kernel_plan_and_rtc_compile(code225):
    """The hypergraph-product kernel (qdec_hgp.cpp): the n = 225 code's Z checks
    factor as [I_12 (x) B | A (x) I_9] with B = A^T (hgp.py homological_product),
    the generated source carries B's and A's edge tables, and hipRTC compiles it
    for gfx950 without a device.  A random matrix, and the same code with two
    columns swapped, are not recognised."""
    import ctypes as C

    from exp_ldpc_amd import _abi
    lib = _abi.load()
    hz = sp.csr_matrix(code225.checks.z)
    h, _, _ = _host_graph(lib, hz, probs=0.01)
    info = (C.c_int32 * 8)()
    assert lib.qd_graph_hgp_info(h, info) == 1
    a0, a1, b0, b1, S, WL, WR, _ = list(info)
    assert (a0, a1, b0, b1) == (12, 9, 9, 12)
    assert S >= 1 and WL == (S * a0 + 63) // 64 and WR == (S * b0 + 63) // 64 and WL + WR <= 16
    L = lib.qd_graph_hgp_source(h, None, 0)
    assert L > 0
    buf = C.create_string_buffer(int(L) + 1)
    assert lib.qd_graph_hgp_source(h, buf, L + 1) == L
    src = buf.value.decode()
    # the factors, as the generator wrote them, rebuild the matrix exactly
    def table(name):
        body = src.split(f"k{name}[")[1].split("{", 1)[1].split("}", 1)[0]
        return [int(t.rstrip("ul")) for t in body.split(",")]
    Brp, Bce, Aer = table("Brp"), table("Bce"), table("Aer")
    assert Brp[-1] == len(Bce) == 36 and len(Aer) == 36
    A = np.zeros((a0, a1), np.uint8)
    B = np.zeros((b0, b1), np.uint8)
    Arp, Bcp = table("Arp"), table("Bcp")
    Arm, Brm = table("Arm"), table("Brm")
    for x in range(a0):
        for w in range(a1):
            A[x, w] = (Arm[x] >> w) & 1
    for y in range(b0):
        for z in range(b1):
            B[y, z] = (Brm[y] >> z) & 1
    H2 = sp.hstack([sp.kron(sp.identity(a0), B), sp.kron(A, sp.identity(b0))]).toarray() % 2
    assert np.array_equal(H2, hz.toarray() % 2)
    assert np.array_equal(A.T, B)  # biregular_hgp: B = A^T
    assert [sum(Arm[x] >> w & 1 for w in range(a1)) for x in range(a0)] == list(np.diff(Arp))
    _abi.check(lib.qd_graph_hgp_compile(h), "hgp compile")  # hipRTC, no device
    # a slot count no workgroup shape holds (2 x 64 x 108 x 16 B of LDS states
    # alone) is refused and the previous plan stays; a feasible one re-plans
    assert lib.qd_graph_hgp_set_slots(h, 64) == -95
    assert lib.qd_graph_hgp_info(h, info) == 1 and list(info)[4] == S
    _abi.check(lib.qd_graph_hgp_set_slots(h, 2), "hgp slots")
    assert lib.qd_graph_hgp_info(h, info) == 1 and list(info)[4] == 2
    assert not hasattr(lib, "qd_graph_hgp_replace_source")  # development builds only
    lib.qd_graph_destroy(h)
    # not hypergraph products
    rng = np.random.default_rng(3)
    R = sp.csr_matrix((rng.random((108, 225)) < 0.03).astype(np.uint8))
    h2, _, _ = _host_graph(lib, R, probs=0.01)
    assert lib.qd_graph_hgp_info(h2, info) == 0
    lib.qd_graph_destroy(h2)
    P = hz.toarray()
    P[:, [0, 150]] = P[:, [150, 0]]
    h3, _, _ = _host_graph(lib, P, probs=0.01)
    assert lib.qd_graph_hgp_info(h3, info) == 0
    lib.qd_graph_destroy(h3)


def test_pack_rows_layout():
    """pack_rows (QD_INPUT_PACKED): bit j of u64 word w = element 64 w + j,
    little-endian bytes, so its bytes equal np.packbits(bitorder='little') of the
    row (Stim's bit_packed rows) zero-padded to 8 bytes; unpack_rows inverts it."""
    from exp_ldpc_amd.decoder import pack_rows, unpack_rows
    rng = np.random.default_rng(4)
    for L in (1, 63, 64, 65, 108, 225, 1000):
        a = rng.integers(0, 2, (5, L)).astype(np.uint8)
        w = pack_rows(a)
        assert w.dtype == np.uint64 and w.shape == (5, (L + 63) // 64)
        for b in range(5):
            for j in range(L):
                assert (int(w[b, j // 64]) >> (j % 64)) & 1 == a[b, j]
        by = w.view(np.uint8)
        pb = np.packbits(a, axis=1, bitorder="little")
        assert np.array_equal(by[:, :pb.shape[1]], pb) and not by[:, pb.shape[1]:].any()
        assert np.array_equal(unpack_rows(w, L), a)


def _m64_model(slot_of, insts):
    """tools/dev/c4_bank_model2.py's cost, the banking gfx950 measured for these
    instructions (tools/dev/lds_atomic_probe.hip): per 64-lane instruction, the
    m1 / m2 reads cost the most lanes on one bank per 32-lane half (slot mod 32),
    the m1 / m2 atomics per 16-lane quarter (slot mod 16), the bit words per
    half ((slot >> 5) mod 32); weights 2 / 2 / 1.5 (operations per edge)."""
    c = 0.0
    for cs in insts:
        s = np.where(cs >= 0, slot_of[np.maximum(cs, 0)], -1)
        for g in range(2):
            h = s[32 * g:32 * g + 32]
            h = h[h >= 0]
            if h.size:
                c += 2.0 * np.bincount(h % 32, minlength=32).max() + 1.5 * np.bincount((h >> 5) % 32).max()
        for g in range(4):
            q = s[16 * g:16 * g + 16]
            q = q[q >= 0]
            if q.size:
                c += 2.0 * np.bincount(q % 16, minlength=16).max()
    return c


def test_lds64_state_slots_spread_the_banks():
    """bp_ms_lds64_kernel's check-state slots (m64_layout) on the C4 code: a
    permutation of the checks whose edge table is the checks' slots, and which
    lowers the bank model of the kernel's per-instruction state accesses by more
    than a quarter against the natural order (the GPU tests pin the decode
    itself)."""
    import ctypes as C

    from exp_ldpc_amd import _abi
    lib = _abi.load()
    hx, hz = load_checks("hgp_80_3_4_s2025")
    H = sp.csr_matrix(hz)
    m, n = H.shape
    h, _, _ = _host_graph(lib, H)
    et = np.zeros(4 * n, np.uint16)
    chk = np.zeros(m, np.uint16)
    _abi.check(lib.qd_graph_lds64_slots_copy(h, _abi.ptr(et), _abi.ptr(chk)), "lds64 slots")
    lib.qd_graph_destroy(h)
    assert np.array_equal(np.sort(chk), np.arange(m))
    slot_of = np.empty(m, np.int64)
    slot_of[chk] = np.arange(m)
    Hc = H.tocsc()
    Hc.sort_indices()
    et = et.reshape(4, n)
    colchk = np.full((4, n), -1)
    for j in range(n):
        rows = Hc.indices[Hc.indptr[j]:Hc.indptr[j + 1]]
        colchk[:rows.size, j] = rows
        assert np.array_equal(et[:rows.size, j], slot_of[rows]) and (et[rows.size:, j] == 0xFFFF).all()
    insts = []
    for w in range(16):
        for r in range((n + 1023) // 1024):
            for k in range(4):
                js = [r * 1024 + ((64 * w + l) * 67) % 1024 for l in range(64)]
                cs = np.array([colchk[k, j] if j < n else -1 for j in js])
                if (cs >= 0).any():
                    insts.append(cs)
    natural = _m64_model(np.arange(m), insts)
    placed = _m64_model(slot_of, insts)
    assert placed < 0.75 * natural, (placed, natural)
