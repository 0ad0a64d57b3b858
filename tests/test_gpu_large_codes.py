"""GPU parity on the larger benchmark codes (BASELINE configs 3-5), built by this
package's own code sources (exp_ldpc_amd/hgp.py, lifted.py):

* C3  [[144,12,12]] bivariate-bicycle lift -> wave kernels, BP + SSF
* C4  biregular_hgp(80,3,4,seed=2025), n = 10^4 (reference-generated fixture)
      -> the LDS-resident kernels (f32 and f64) and the HBM-message workgroup /
      slot-group kernels, BP + SSF
* C5  as BASELINE names it: the PSL(2,16) Cayley-graph lifted-product code
      lifted_product_code_pgl2(1, 4, 2, double_cover=False, seed=1), n = 53,040,
      k = 4080 (fixture tests/golden/lp_pgl2_1_4_2_s1_*): BP + SSF + logical check
      at R = 0, and the R = 1 spacetime graph (48,960 x 130,560) with fold +
      logical check, on the slot-group kernel (the default for graphs whose
      messages spill to HBM) and on the workgroup kernel
* extra graphs: PSL(2,q) matrix lifts, q = 5 (n = 2700) and q = 13 (n = 49,140)

Every output is compared bit-for-bit with the CPU oracle on the same sampled
storage-experiment shots (min-sum LLRs within the fp tolerance of
test_gpu_parity._cmp_llr)."""
import numpy as np
import pytest
import scipy.sparse as sp

from exp_ldpc_amd import decoder

from conftest import load_checks

pytestmark = pytest.mark.gpu

SEED = 20250221
KEYS_SSF = ("x", "corr", "iters", "status", "ssf_steps", "fail")


def _decode_both(oracle_lib, H, prior, syn, *, rd=None, gens=None, lz=None, max_iter=50, method="ms",
                 precision="f32", keys=("x", "iters", "status"), **kw):
    from exp_ldpc_amd.decoder import Decoder
    dec = Decoder(H, prior, method=method, precision=precision, max_iter=max_iter, flip_sets=gens, logicals=lz, **kw)
    got = dec.decode(syn, readout=rd, want=keys)
    ref = oracle_lib.decode(H, prior, syn, method=method, precision=precision, max_iter=max_iter,
                            ssf=gens is not None, gens=gens, lz=lz, readout=rd, want_llr=False,
                            ssf_impl="fast", **kw)
    for k in keys:
        assert np.array_equal(got[k], ref[k]), k
    return got


@pytest.fixture(scope="module")
def bb144():
    from exp_ldpc_amd.lifted import bivariate_bicycle_code
    return bivariate_bicycle_code(12, 6, [(3, 0), (0, 1), (0, 2)], [(0, 3), (1, 0), (2, 0)], compute_logicals=True)


@pytest.mark.parametrize("p", [0.003, 0.01, 0.03])
def test_bb144_bp_ssf_parity(gpu_available, oracle_lib, bb144, p):
    hx, hz, lz = bb144.checks.x, bb144.checks.z, bb144.logicals.z
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=SEED, stream=3, shot0=0, B=3000)
    got = _decode_both(oracle_lib, hz, 2 * p / 3, syn, rd=rd, gens=hx, lz=lz, keys=KEYS_SSF)
    if p >= 0.01:
        assert (got["status"] & 1).mean() < 1.0  # BP failures reach SSF


def test_bb144_device_sampler_matches_oracle(gpu_available, oracle_lib, bb144):
    import torch
    from exp_ldpc_amd.decoder import Decoder
    hz = bb144.checks.z
    B = 4096
    dec = Decoder(hz, 0.01, method="ms", precision="f32", max_iter=50)
    syn = torch.empty((B, hz.shape[0]), dtype=torch.uint8, device="cuda:0")
    rd = torch.empty((B, hz.shape[1]), dtype=torch.uint8, device="cuda:0")
    dec.sample_storage_device(0, 0.02, 0.02, SEED, 1, 12345, B, syn, rd)
    torch.cuda.synchronize()
    rs, rr = oracle_lib.sample_storage(hz, 0, 0.02, 0.02, seed=SEED, stream=1, shot0=12345, B=B)
    assert np.array_equal(syn.cpu().numpy(), rs) and np.array_equal(rd.cpu().numpy(), rr)


@pytest.fixture(scope="module")
def hgp10k():
    from exp_ldpc_amd import gf2
    hx, hz = load_checks("hgp_80_3_4_s2025")
    _, lz = gf2.css_logicals(hx, hz)
    return hx, hz, lz


def test_hgp10k_bp_ssf_parity(gpu_available, oracle_lib, hgp10k):
    hx, hz, lz = hgp10k
    assert hz.shape == (4800, 10000) and lz.shape[0] == 400
    p = 0.03
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=SEED, stream=4, shot0=0, B=192)
    got = _decode_both(oracle_lib, hz, 2 * p / 3, syn, rd=rd, gens=hx, lz=lz, max_iter=30, keys=KEYS_SSF)
    assert got["ssf_steps"].sum() > 0


def test_hgp10k_group_kernel_forced_parity(gpu_available, oracle_lib, hgp10k, monkeypatch):
    """The slot-group HBM-streaming kernel forced (QD_OPT_GROUP_KERNEL = 1) on C4 in
    fp32, where the LDS-resident kernel is the default."""
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "group_kernel", 1)
    hx, hz, lz = hgp10k
    p = 0.03
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=SEED, stream=9, shot0=0, B=160)
    got = _decode_both(oracle_lib, hz, 2 * p / 3, syn, rd=rd, gens=hx, lz=lz, max_iter=30, keys=KEYS_SSF)
    assert got["ssf_steps"].sum() > 0


@pytest.mark.parametrize("kernel", ["auto", "group"])
@pytest.mark.parametrize("p", [0.01, 0.03])
def test_hgp10k_f64_bp_ssf_fail_parity(gpu_available, oracle_lib, hgp10k, p, kernel, monkeypatch):
    """C4 at ldpc's precision: BP min-sum f64 max_iter 50 (auto: the LDS-resident
    bp_ms_lds64_kernel; group: the slot-group kernel, messages in HBM, with
    QD_OPT_LDS_KERNEL = 0) + SSF + logical check, 256 sampled shots, bit-exact."""
    if kernel == "group":
        monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "lds_kernel", 0)
    hx, hz, lz = hgp10k
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=SEED, stream=14, shot0=0, B=256)
    got = _decode_both(oracle_lib, hz, 2 * p / 3, syn, rd=rd, gens=hx, lz=lz, max_iter=50, precision="f64",
                       keys=KEYS_SSF)
    if p >= 0.03:
        assert (got["status"] & 1).mean() < 0.9 and got["ssf_steps"].sum() > 0


def test_hgp10k_bp_f64_llr(gpu_available, oracle_lib, hgp10k):
    from test_gpu_parity import _cmp_llr
    from exp_ldpc_amd.decoder import Decoder
    _, hz, _ = hgp10k
    syn, _ = oracle_lib.sample_storage(hz, 0, 0.02, 0.02, seed=SEED, stream=5, shot0=0, B=96)
    for method, precision in (("ms", "f64"), ("ps", "f64")):
        dec = Decoder(hz, 0.0133, method=method, precision=precision, max_iter=20)
        got = dec.decode(syn, want=("x", "llr", "iters", "status"))
        ref = oracle_lib.decode(hz, 0.0133, syn, method=method, precision=precision, max_iter=20)
        for k in ("x", "iters", "status"):
            assert np.array_equal(got[k], ref[k]), (method, k)
        _cmp_llr(got["llr"], ref["llr"], method, precision)


@pytest.fixture(scope="module")
def psl5():
    from exp_ldpc_amd.lifted import psl2_lifted_product_code
    return psl2_lifted_product_code(5, compute_logicals=True)


def test_psl5_lift_bp_parity(gpu_available, oracle_lib, psl5):
    hz, lz = psl5.checks.z, psl5.logicals.z
    p = 0.02
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=SEED, stream=6, shot0=0, B=400)
    _decode_both(oracle_lib, hz, 2 * p / 3, syn, rd=rd, lz=lz, max_iter=40, keys=("x", "corr", "iters", "status", "fail"))


@pytest.fixture(scope="module")
def psl13_hz():
    from exp_ldpc_amd.lifted import psl2_lifted_product_code
    return psl2_lifted_product_code(13).checks.z


def test_psl13_lift_bp_parity(gpu_available, oracle_lib, psl13_hz):
    hz = psl13_hz
    assert hz.shape[1] == 49140
    p = 0.01
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=SEED, stream=7, shot0=0, B=48)
    _decode_both(oracle_lib, hz, 2 * p / 3, syn, max_iter=15)


@pytest.mark.parametrize("kernel", ["workgroup", "group"])
def test_psl13_lift_spacetime_r1_parity(gpu_available, oracle_lib, psl13_hz, kernel, monkeypatch):
    """The PSL(2,13) matrix lift's multi-round spacetime syndromes: H_st =
    [blockdiag(Hz, Hz) | M] (spacetime_code.py:46-75), sampled by the
    storage-experiment sampler at R = 1 and folded onto the data qubits; both
    HBM-message kernels."""
    from exp_ldpc_amd.spacetime import SpacetimeCode
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "group_kernel", 1 if kernel == "group" else 0)
    hz = psl13_hz
    H = sp.csr_matrix(SpacetimeCode(hz, 1).spacetime_check_matrix)
    p = 0.005
    syn, rd = oracle_lib.sample_storage(hz, 1, p, p, seed=SEED, stream=8, shot0=0, B=24)
    _decode_both(oracle_lib, H, 2 * p / 3, syn, max_iter=10, keys=("corr", "iters", "status"),
                 n_data=hz.shape[1], fold_blocks=2)


def test_psl13_spacetime_r1_product_sum_f32(gpu_available, oracle_lib, psl13_hz):
    """Product-sum f32 on the placement-0 graph (shot state in HBM, hard-decision
    bits in LDS): the reference CLI default bp_method with the p_sweep-style f32
    variant, x / iterations / status bit-exact, corrections folded at R = 1."""
    from exp_ldpc_amd.spacetime import SpacetimeCode
    hz = psl13_hz
    H = sp.csr_matrix(SpacetimeCode(hz, 1).spacetime_check_matrix)
    p = 0.005
    syn, rd = oracle_lib.sample_storage(hz, 1, p, p, seed=SEED, stream=9, shot0=0, B=12)
    _decode_both(oracle_lib, H, 2 * p / 3, syn, max_iter=8, method="ps", precision="f32",
                 keys=("x", "corr", "iters", "status"), n_data=hz.shape[1], fold_blocks=2)


@pytest.mark.parametrize("p", [0.01, 0.03, 0.06])
def test_hgp10k_lds_kernel_parity(gpu_available, oracle_lib, hgp10k, p):
    """C4 on the LDS-resident min-sum kernel (bp_ms_lds_kernel, the default for
    fp32 min-sum on this graph): hard decisions, iteration counts, SSF steps,
    corrections and failure flags bit-exact at low, medium and high p (the last
    one runs most shots to max_iter)."""
    hx, hz, lz = hgp10k
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=SEED, stream=11, shot0=0, B=256)
    got = _decode_both(oracle_lib, hz, 2 * p / 3, syn, rd=rd, gens=hx, lz=lz, max_iter=50, keys=KEYS_SSF)
    if p >= 0.03:
        assert (got["status"] & 1).mean() < 0.9 and got["ssf_steps"].sum() > 0


def test_hgp10k_workgroup_kernel_parity(gpu_available, oracle_lib, hgp10k, monkeypatch):
    """The HBM-message workgroup kernel stays covered on C4 (QD_OPT_LDS_KERNEL = 0,
    QD_OPT_GROUP_KERNEL = 0)."""
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "lds_kernel", 0)
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "group_kernel", 0)
    hx, hz, lz = hgp10k
    p = 0.03
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=SEED, stream=12, shot0=0, B=96)
    _decode_both(oracle_lib, hz, 2 * p / 3, syn, rd=rd, gens=hx, lz=lz, max_iter=30, keys=KEYS_SSF)


@pytest.mark.parametrize("seed", [3, 4])
def test_lds_kernel_random_irregular(gpu_available, oracle_lib, seed, monkeypatch):
    """bp_ms_lds_kernel forced (QD_OPT_LDS_KERNEL = 1) on ragged graphs outside the wave
    shapes: check degrees 0..8 (empty and single-edge rows), variable degrees
    0..4, per-column priors, ms_scaling both ways; x / iterations / status."""
    from exp_ldpc_amd.codes import make_check_matrix
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "lds_kernel", 1)
    rng = np.random.default_rng(seed)
    m, n = int(rng.integers(600, 1500)), int(rng.integers(700, 3000))
    rows, colcount = [], np.zeros(n, int)
    for i in range(m):
        d = int(rng.integers(0, 9))
        cand = [j for j in rng.permutation(n) if colcount[j] < 4][:d]
        for j in cand:
            colcount[j] += 1
        rows.append(sorted(cand))
    H = make_check_matrix(rows, n)
    e = (rng.random((300, n)) < 0.02).astype(np.uint8)
    syn = ((H @ e.T).T % 2).astype(np.uint8)
    probs = rng.uniform(0.005, 0.1, n)
    for scaling in (0.0, 0.625):
        _decode_both(oracle_lib, H, probs, syn, max_iter=30, ms_scaling=scaling)
    # iteration 1 comes from the launch's image (no check pass): 1 and 2 iterations
    for mi in (1, 2):
        _decode_both(oracle_lib, H, probs, syn, max_iter=mi, ms_scaling=0.625 if mi == 2 else 0.0)


def test_lds_kernel_zero_and_negative_priors(gpu_available, oracle_lib, monkeypatch):
    """bp_ms_lds_kernel's sign-bit check pass on messages that are exactly zero
    (columns with p = 0.5: prior LLR +0, so +0 v2c messages and -0 c2v ones)
    and negative (p > 0.5), beside ordinary columns: x / iterations / status
    bit-exact against the oracle's compares."""
    from exp_ldpc_amd.codes import make_check_matrix
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "lds_kernel", 1)
    rng = np.random.default_rng(5)
    m, n = 900, 1600
    rows, colcount = [], np.zeros(n, int)
    for i in range(m):
        d = int(rng.integers(2, 9))
        cand = [j for j in rng.permutation(n) if colcount[j] < 4][:d]
        for j in cand:
            colcount[j] += 1
        rows.append(sorted(cand))
    H = make_check_matrix(rows, n)
    e = (rng.random((300, n)) < 0.03).astype(np.uint8)
    syn = ((H @ e.T).T % 2).astype(np.uint8)
    probs = rng.choice([0.5, 0.5, 0.6, 0.02, 0.05, 0.01], n)
    for scaling in (0.0, 0.625):
        _decode_both(oracle_lib, H, probs, syn, max_iter=20, ms_scaling=scaling)


def _decode_lds64(oracle_lib, H, prior, syn, **kw):
    """_decode_both at f64 with bp_ms_lds64_kernel forced; asserts it ran."""
    from exp_ldpc_amd.decoder import Decoder
    keys = kw.pop("keys", ("x", "iters", "status"))
    rd, gens, lz = kw.pop("rd", None), kw.pop("gens", None), kw.pop("lz", None)
    max_iter = kw.pop("max_iter", 50)
    dec = Decoder(H, prior, method="ms", precision="f64", max_iter=max_iter, flip_sets=gens, logicals=lz, **kw)
    got = dec.decode(syn, readout=rd, want=keys)
    assert "bp_ms_lds64_kernel" in dec.last_kernels()[0]
    ref = oracle_lib.decode(H, prior, syn, method="ms", precision="f64", max_iter=max_iter, ssf=gens is not None,
                            gens=gens, lz=lz, readout=rd, want_llr=False, ssf_impl="fast", **kw)
    for k in keys:
        assert np.array_equal(got[k], ref[k]), k
    return got


@pytest.mark.parametrize("p", [0.005, 0.03, 0.06])
def test_hgp10k_lds64_kernel_parity(gpu_available, oracle_lib, hgp10k, p, monkeypatch):
    """C4 at ldpc's precision on the LDS-resident f64 kernel (bp_ms_lds64_kernel:
    v2c messages in registers, check states by LDS atomics; QD_OPT_LDS_KERNEL = 1):
    x / corrections / iterations / status / SSF steps / failure flags bit-exact,
    low to high p (the last runs most shots to max_iter)."""
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "lds_kernel", 1)
    hx, hz, lz = hgp10k
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=SEED, stream=15, shot0=0, B=256)
    got = _decode_lds64(oracle_lib, hz, 2 * p / 3, syn, rd=rd, gens=hx, lz=lz, max_iter=50, keys=KEYS_SSF)
    if p >= 0.03:
        assert (got["status"] & 1).mean() < 0.9 and got["ssf_steps"].sum() > 0


@pytest.mark.parametrize("seed", [3, 4])
def test_lds64_kernel_random_irregular(gpu_available, oracle_lib, seed, monkeypatch):
    """bp_ms_lds64_kernel on ragged graphs: check degrees 0..8 (empty and
    single-edge rows: m2 stays Big), variable degrees 0..4, per-column priors,
    ms_scaling both ways, max_iter 1 and 30; x / iterations / status."""
    from exp_ldpc_amd.codes import make_check_matrix
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "lds_kernel", 1)
    rng = np.random.default_rng(seed)
    m, n = int(rng.integers(600, 1500)), int(rng.integers(700, 3000))
    rows, colcount = [], np.zeros(n, int)
    for i in range(m):
        d = int(rng.integers(0, 9))
        cand = [j for j in rng.permutation(n) if colcount[j] < 4][:d]
        for j in cand:
            colcount[j] += 1
        rows.append(sorted(cand))
    H = make_check_matrix(rows, n)
    e = (rng.random((300, n)) < 0.02).astype(np.uint8)
    syn = ((H @ e.T).T % 2).astype(np.uint8)
    probs = rng.uniform(0.005, 0.1, n)
    for scaling in (0.0, 0.625):
        _decode_lds64(oracle_lib, H, probs, syn, max_iter=30, ms_scaling=scaling)
    _decode_lds64(oracle_lib, H, probs, syn, max_iter=1)


@pytest.mark.parametrize("n,m,n3,inst", [(8000, 4000, 4500, "<8, 4>"), (7000, 4000, 0, "<8, 0>"),
                                          (9800, 4800, 3500, "<10, 3>"), (9300, 4900, 0, "<10, 0>")])
def test_lds64_kernel_degree3_rounds(gpu_available, oracle_lib, n, m, n3, inst, monkeypatch):
    """bp_ms_lds64_kernel's D3R instantiations (leading 1024-column rounds whose
    columns all have degree <= 3 keep 3 messages in registers): columns j < n3
    of degree 3, the rest of degree 4, so the host's count picks the
    instantiation asserted; x / iterations / status bit-exact."""
    from exp_ldpc_amd.codes import make_check_matrix
    from exp_ldpc_amd.decoder import Decoder
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "lds_kernel", 1)
    rng = np.random.default_rng(n)
    rows, cnt = [[] for _ in range(m)], np.zeros(m, int)
    for j in range(n):  # row degrees <= 8 (the kernel's check-row bound)
        for i in rng.choice(np.flatnonzero(cnt < 8), 3 if j < n3 else 4, replace=False):
            rows[i].append(j)
            cnt[i] += 1
    H = make_check_matrix([sorted(r) for r in rows], n)
    e = (rng.random((96, n)) < 0.01).astype(np.uint8)
    syn = ((H @ e.T).T % 2).astype(np.uint8)
    probs = rng.uniform(0.005, 0.03, n)
    _decode_lds64(oracle_lib, H, probs, syn, max_iter=30)
    dec = Decoder(H, probs, method="ms", precision="f64", max_iter=30)
    dec.decode(syn[:4], want=("x",))
    assert dec.last_kernels()[0].startswith("qdec::bp_ms_lds64_kernel" + inst), dec.last_kernels()


def test_lds64_kernel_zero_and_negative_priors(gpu_available, oracle_lib, monkeypatch):
    """bp_ms_lds64_kernel on exactly-zero messages (p = 0.5 columns: +0 priors,
    ties at m1 = 0, -0 c2v) and negative priors (p > 0.5)."""
    from exp_ldpc_amd.codes import make_check_matrix
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "lds_kernel", 1)
    rng = np.random.default_rng(5)
    m, n = 900, 1600
    rows, colcount = [], np.zeros(n, int)
    for i in range(m):
        d = int(rng.integers(2, 9))
        cand = [j for j in rng.permutation(n) if colcount[j] < 4][:d]
        for j in cand:
            colcount[j] += 1
        rows.append(sorted(cand))
    H = make_check_matrix(rows, n)
    e = (rng.random((300, n)) < 0.03).astype(np.uint8)
    syn = ((H @ e.T).T % 2).astype(np.uint8)
    probs = rng.choice([0.5, 0.5, 0.6, 0.02, 0.05, 0.01], n)
    for scaling in (0.0, 0.625):
        _decode_lds64(oracle_lib, H, probs, syn, max_iter=20, ms_scaling=scaling)


@pytest.mark.parametrize("scoring", ["auto", "scan"])
def test_hgp10k_ssf_table_scoring_parity(gpu_available, oracle_lib, hgp10k, scoring, monkeypatch):
    """The incremental workgroup SSF kernel scores generators by table lookup
    when the graph's score tables qualify (every generator of this HGP code
    shares one 4096-entry table; QD_SSF_AUTO) or by the subset search
    (QD_SSF_SCAN): both equal the oracle, f32 and f64."""
    from exp_ldpc_amd.decoder import Decoder
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "ssf", scoring)
    hx, hz, lz = hgp10k
    d = Decoder(hz, 0.02, method="ms", precision="f32", max_iter=5, flip_sets=hx)
    assert d.ssf_tables() == (True, 4096 * 4)  # score tables only (beyond the wave shapes)
    assert d.get_option("ssf") == (0 if scoring == "auto" else 1)
    p = 0.03
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=SEED, stream=17, shot0=0, B=128)
    for precision in ("f32", "f64"):
        got = _decode_both(oracle_lib, hz, 2 * p / 3, syn, rd=rd, gens=hx, lz=lz, max_iter=30, keys=KEYS_SSF,
                           precision=precision)
        assert got["ssf_steps"].sum() > 0


def test_hgp10k_ssf_rescan_kernel_parity(gpu_available, oracle_lib, hgp10k, monkeypatch):
    """The re-scanning SSF block kernel (QD_OPT_SSF_INC = 0) stays covered; the
    default incremental one is covered by every other C4 test."""
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "ssf_inc", 0)
    hx, hz, lz = hgp10k
    p = 0.03
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=SEED, stream=13, shot0=0, B=96)
    got = _decode_both(oracle_lib, hz, 2 * p / 3, syn, rd=rd, gens=hx, lz=lz, max_iter=30, keys=KEYS_SSF)
    assert got["ssf_steps"].sum() > 0


# ------------------------------------------------------------------ config 5 as named
@pytest.fixture(scope="module")
def c5():
    """BASELINE config 5: the PSL(2,16) Cayley-graph LP code (checks and
    logicals from the committed fixture, tools/fixtures/make_c5_fixture.py)."""
    from conftest import load_logicals
    hx, hz = load_checks("lp_pgl2_1_4_2_s1")
    _, lz = load_logicals("lp_pgl2_1_4_2_s1")
    assert hz.shape == (24480, 53040) and lz.shape == (4080, 53040)
    return hx, hz, lz


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("kernel", ["group", "workgroup"])
def test_c5_r0_bp_ssf_fail_parity(gpu_available, oracle_lib, c5, precision, kernel, monkeypatch):
    """Config 5 at R = 0: BP min-sum (max_iter 50) + SSF on the Hx flip sets +
    logical check, 256 sampled shots, every output bit-exact."""
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "group_kernel", 1 if kernel == "group" else 0)
    hx, hz, lz = c5
    p = 0.004
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=SEED, stream=21, shot0=0, B=256)
    got = _decode_both(oracle_lib, hz, 2 * p / 3, syn, rd=rd, gens=hx, lz=lz, precision=precision, keys=KEYS_SSF)
    assert (got["status"] & 1).mean() < 1.0 and got["ssf_steps"].sum() > 0


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_c5_spacetime_r1_fold_fail_parity(gpu_available, oracle_lib, c5, precision):
    """Config 5's multi-round spacetime syndromes: R = 1 (H_st 48,960 x 130,560,
    spacetime_code.py:46-75), BP min-sum max_iter 50, corrections folded onto the
    data qubits and the logical check, 256 shots, on the slot-group kernel."""
    from exp_ldpc_amd.spacetime import SpacetimeCode
    _, hz, lz = c5
    H = sp.csr_matrix(SpacetimeCode(hz, 1).spacetime_check_matrix)
    assert H.shape == (48960, 130560)
    p = 0.002
    syn, rd = oracle_lib.sample_storage(hz, 1, p, p, seed=SEED, stream=22, shot0=0, B=256)
    got = _decode_both(oracle_lib, H, 2 * p / 3, syn, rd=rd, lz=lz, precision=precision,
                       keys=("x", "corr", "iters", "status", "fail"), n_data=hz.shape[1], fold_blocks=2)
    assert 0 < got["fail"].sum() < 256 or (got["status"] & 1).all()


def test_c5_spacetime_r1_product_sum_f64(gpu_available, oracle_lib, c5):
    """Product-sum (the reference CLI's default bp_method) in f64 on config 5's
    R = 1 spacetime graph, slot-group kernel: x, folded corrections, iterations,
    status and failure flags bit-exact."""
    from exp_ldpc_amd.spacetime import SpacetimeCode
    _, hz, lz = c5
    H = sp.csr_matrix(SpacetimeCode(hz, 1).spacetime_check_matrix)
    p = 0.002
    syn, rd = oracle_lib.sample_storage(hz, 1, p, p, seed=SEED, stream=23, shot0=0, B=128)
    _decode_both(oracle_lib, H, 2 * p / 3, syn, rd=rd, lz=lz, method="ps", precision="f64", max_iter=30,
                 keys=("x", "corr", "iters", "status", "fail"), n_data=hz.shape[1], fold_blocks=2)


def test_group_kernel_llr_and_ragged(gpu_available, oracle_lib, monkeypatch):
    """The slot-group kernel forced on a ragged random graph (check degrees 0..9,
    column degrees 0..5, per-column priors): min-sum and product-sum, f32 and
    f64, with more shots than slots so slots are refilled mid-flight; x,
    iterations, status and LLRs (min-sum exact, product-sum within the device
    log tolerance)."""
    from test_gpu_parity import _cmp_llr
    from exp_ldpc_amd.codes import make_check_matrix
    from exp_ldpc_amd.decoder import Decoder
    monkeypatch.setitem(decoder.DEFAULT_OPTIONS, "group_kernel", 1)
    rng = np.random.default_rng(17)
    m, n = 700, 1500
    rows, colcount = [], np.zeros(n, int)
    for i in range(m):
        d = int(rng.integers(0, 10))
        cand = [j for j in rng.permutation(n) if colcount[j] < 5][:d]
        for j in cand:
            colcount[j] += 1
        rows.append(sorted(cand))
    H = make_check_matrix(rows, n)
    e = (rng.random((700, n)) < 0.03).astype(np.uint8)
    syn = ((H @ e.T).T % 2).astype(np.uint8)
    probs = rng.uniform(0.01, 0.08, n)
    for method in ("ms", "ps"):
        for precision in ("f32", "f64"):
            dec = Decoder(H, probs, method=method, precision=precision, max_iter=25)
            got = dec.decode(syn, want=("x", "llr", "iters", "status"))
            ref = oracle_lib.decode(H, probs, syn, method=method, precision=precision, max_iter=25)
            for k in ("x", "iters", "status"):
                assert np.array_equal(got[k], ref[k]), (method, precision, k)
            _cmp_llr(got["llr"], ref["llr"], method, precision)
            # fewer shots than one group's 64 slots (idle slots from the start)
            small = dec.decode(syn[:5], want=("x", "iters", "status"))
            for k in ("x", "iters", "status"):
                assert np.array_equal(small[k], ref[k][:5]), (method, precision, "B=5", k)


def test_c5_run_simulation_bpssf_matches_oracle(gpu_available, oracle_lib, c5):
    """The harness end to end on config 5 (reference run_simulation with
    BPSSFCorrect, R = 0): the code carries its 4080 logicals as sparse CSR
    (codes.QuantumCodeLogicals), shots come from the device sampler, and the
    per-shot failure flags equal the CPU oracle's on the same Philox shots."""
    from exp_ldpc_amd.codes import QuantumCode, QuantumCodeChecks, QuantumCodeLogicals
    from exp_ldpc_amd.experiment import run_simulation
    from exp_ldpc_amd.noise_model import depolarizing_noise
    from conftest import load_logicals
    hx, hz, lz = c5
    lx, _ = load_logicals("lp_pgl2_1_4_2_s1")
    code = QuantumCode(QuantumCodeChecks(hx, hz), QuantumCodeLogicals(lx, lz))
    opts = {"max_iter": 50, "bp_method": "ms", "ms_scaling_factor": 0, "osd_method": "osd0", "osd_order": 0}
    p = 0.004
    pr = 2 * p / 3
    fails = run_simulation(256, code, lambda a, b: pr, lambda a, b: pr, depolarizing_noise, {"p": p, "pm": p}, opts,
                           0, "bpssf", seed=3, batch=256, precision="f64")
    syn, rd = oracle_lib.sample_storage(hz, 0, p, p, seed=3, stream=0, shot0=0, B=256)
    ref = oracle_lib.decode(hz, pr, syn, method="ms", precision="f64", max_iter=50, ssf=True, gens=hx, lz=lz,
                            readout=rd, want_llr=False, ssf_impl="fast")
    assert np.array_equal(fails, ref["fail"].astype(bool))
