"""Bit-packed device inputs (QD_INPUT_PACKED, include/qdec.h; SURVEY §8(b)'s
"optionally bit-packed" syndrome / readout flag).  The reference's sampler is
Stim's compile_sampler().sample (python/qldpc/misc/_experiment.py:196-197),
whose bit_packed=True rows are the same little-endian bits this layout holds.

Checked here, every comparison byte for byte:
  * the packed sampler writes pack_rows(the byte sampler's rows) == the oracle's
    rows packed, at R = 0..3;
  * packed decode == byte decode == the oracle on the benchmarked call (lean
    min-sum + SSF + fused failure check, the two-pass path whose triage reads
    the words directly) at all 9 sweep points, f64 and f32;
  * packed decode on paths that expand the words first (x / llr outputs,
    product-sum, syndrome flags with base and readout, the host-buffer entry
    point, a workgroup-kernel graph) equals the byte decode;
  * ragged batches (1, 63, 65 shots) and padding bits set in the words."""
import numpy as np
import pytest

from conftest import load_checks, load_code

pytestmark = pytest.mark.gpu

SEED = 20250221


def _sample_both(dec, rounds, p, stream_id, shot0, B, m, n):
    import torch
    syn = torch.empty((B, (rounds + 1) * m), dtype=torch.uint8, device="cuda")
    rd = torch.empty((B, n), dtype=torch.uint8, device="cuda")
    sw = torch.empty((B, ((rounds + 1) * m + 63) // 64), dtype=torch.int64, device="cuda")
    rw = torch.empty((B, (n + 63) // 64), dtype=torch.int64, device="cuda")
    dec.sample_storage_device(rounds, p, p, SEED, stream_id, shot0, B, syn, rd)
    dec.sample_storage_device(rounds, p, p, SEED, stream_id, shot0, B, sw, rw, packed=True)
    torch.cuda.synchronize()
    return syn, rd, sw, rw


@pytest.mark.parametrize("rounds", [0, 1, 2, 3])
def test_packed_sampler_equals_packed_bytes(gpu_available, oracle_lib, rounds):
    from exp_ldpc_amd.decoder import Decoder, pack_rows
    hx, hz = load_checks("hgp_12_3_4_s1234")
    m, n = hz.shape
    dec = Decoder(hz, 0.01)
    B = 1000
    syn, rd, sw, rw = _sample_both(dec, rounds, 0.03, 7, 999, B, m, n)
    rs, rr = oracle_lib.sample_storage(hz, rounds, 0.03, 0.03, seed=SEED, stream=7, shot0=999, B=B)
    assert np.array_equal(syn.cpu().numpy(), rs) and np.array_equal(rd.cpu().numpy(), rr)
    assert np.array_equal(sw.cpu().numpy().view(np.uint64), pack_rows(rs))
    assert np.array_equal(rw.cpu().numpy().view(np.uint64), pack_rows(rr))


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_packed_bench_call_all_points(gpu_available, oracle_lib, precision):
    """bench.py's decode (syn + readout in; iters, status, ssf_steps, fail out)
    on packed rows: the triage reads the words (the two-pass path runs), and
    every output equals the byte-row decode and the oracle."""
    import torch
    from exp_ldpc_amd.decoder import Decoder
    code = load_code("hgp_12_3_4_s1234")
    hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
    m, n = hz.shape
    B = 4096
    for pi, p in enumerate(np.geomspace(1e-3, 1e-1, 9)):
        dec = Decoder(hz, 2 * p / 3, method="ms", precision=precision, max_iter=50, ms_scaling=0.0, flip_sets=hx,
                      logicals=lz)
        syn, rd, sw, rw = _sample_both(dec, 0, p, pi, 5 << 18, B, m, n)
        outs = []
        for packed in (False, True):
            o = {k: torch.empty(B, dtype=dt, device="cuda") for k, dt in
                 (("iters", torch.int32), ("status", torch.uint8), ("ssf_steps", torch.int32), ("fail", torch.uint8))}
            dec.decode_device(B, syn=sw if packed else syn, readout=rw if packed else rd, packed=packed, **o)
            torch.cuda.synchronize()
            bp_k, _, pre_k = dec.last_kernels()
            assert "cmp_kernel" in bp_k and "triage" in pre_k, (bp_k, pre_k)
            outs.append({k: v.cpu().numpy() for k, v in o.items()})
        ref = oracle_lib.decode(hz, 2 * p / 3, syn.cpu().numpy(), method="ms", precision=precision, max_iter=50,
                                ssf=True, gens=hx, lz=lz, readout=rd.cpu().numpy(), want_llr=False, ssf_impl="fast")
        for k in outs[0]:
            assert np.array_equal(outs[1][k], outs[0][k]), (p, k)
            assert np.array_equal(outs[1][k], ref[k]), (p, k)


@pytest.mark.parametrize("B", [1, 63, 65, 3000])
def test_packed_ragged_batches_and_padding_bits(gpu_available, oracle_lib, B):
    """Padding bits of the last word are ignored (set here on purpose), and
    batches that end inside a 64-shot triage tile decode like the byte rows."""
    import torch
    from exp_ldpc_amd.decoder import Decoder, pack_rows
    code = load_code("hgp_12_3_4_s1234")
    hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
    m, n = hz.shape
    rng = np.random.default_rng(B)
    rr = (rng.random((B, n)) < 0.02).astype(np.uint8)
    rs = np.ascontiguousarray(((hz @ ((rr ^ (rng.random((B, n)) < 0.01)).T)).T % 2).astype(np.uint8))
    sw, rw = pack_rows(rs), pack_rows(rr)
    sw[:, -1] |= np.uint64(0xFFFF) << np.uint64(m % 64)   # m = 108: bits 44..59 are padding
    rw[:, -1] |= np.uint64(1) << np.uint64(63)            # n = 225: bit 63 of word 3 is padding
    dec = Decoder(hz, 0.02, method="ms", precision="f64", max_iter=50, flip_sets=hx, logicals=lz)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda")
    res = []
    for packed in (False, True):
        o = {k: torch.empty(B, dtype=dt, device="cuda") for k, dt in
             (("iters", torch.int32), ("status", torch.uint8), ("ssf_steps", torch.int32), ("fail", torch.uint8))}
        if packed:
            dec.decode_device(B, syn=t(sw), readout=t(rw), packed=True, **o)
        else:
            dec.decode_device(B, syn=torch.from_numpy(rs).to("cuda"), readout=torch.from_numpy(rr).to("cuda"), **o)
        torch.cuda.synchronize()
        res.append({k: v.cpu().numpy() for k, v in o.items()})
    for k in res[0]:
        assert np.array_equal(res[0][k], res[1][k]), k


def test_packed_inputs_on_expanding_paths(gpu_available, oracle_lib):
    """Calls off the two-pass path expand the words first (unpack_rows_kernel):
    x / llr outputs, product-sum, syndrome flags with base + readout, the host
    entry point, and the n = 10^4 workgroup graph (C4 code)."""
    import torch
    from exp_ldpc_amd.decoder import Decoder, pack_rows
    code = load_code("hgp_12_3_4_s1234")
    hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
    m, n = hz.shape
    rng = np.random.default_rng(5)
    B = 700
    rr = (rng.random((B, n)) < 0.03).astype(np.uint8)
    base = (rng.random((B, n)) < 0.01).astype(np.uint8)
    rs = np.ascontiguousarray(((hz @ rr.T).T % 2).astype(np.uint8))
    want = ("x", "corr", "llr", "iters", "status", "ssf_steps", "fail")
    for method in ("ms", "ps"):
        dec = Decoder(hz, 0.02, method=method, precision="f64", max_iter=30, flip_sets=hx, logicals=lz)
        a = dec.decode(rs, readout=rr, want=want)
        b = dec.decode(pack_rows(rs), readout=pack_rows(rr), want=want, packed=True)
        for k in want:
            assert np.array_equal(a[k], b[k]), (method, k)
        # syndrome from base ^ readout (flags 3), no explicit syndrome
        a = dec.decode(None, base=base, readout=rr, syn_flags=3, want=want)
        b = dec.decode(None, base=pack_rows(base), readout=pack_rows(rr), syn_flags=3, want=want, packed=True)
        for k in want:
            assert np.array_equal(a[k], b[k]), (method, "flags", k)
    # device buffers with an x output (one-pass wave kernel after the expansion)
    dec = Decoder(hz, 0.02, method="ms", precision="f32", max_iter=30, flip_sets=hx, logicals=lz)
    t = lambda v: torch.from_numpy(np.ascontiguousarray(v)).to("cuda")
    xs = [torch.empty((B, n), dtype=torch.uint8, device="cuda") for _ in range(2)]
    fs = [torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(2)]
    dec.decode_device(B, syn=t(rs), readout=t(rr), x=xs[0], fail=fs[0])
    dec.decode_device(B, syn=t(pack_rows(rs).view(np.int64)), readout=t(pack_rows(rr).view(np.int64)), x=xs[1],
                      fail=fs[1], packed=True)
    torch.cuda.synchronize()
    assert torch.equal(xs[0], xs[1]) and torch.equal(fs[0], fs[1])
    # workgroup graph (C4 code): expansion, then the LDS-resident kernel
    hx4, hz4 = load_checks("hgp_80_3_4_s2025")
    dec4 = Decoder(hz4, 0.01, method="ms", precision="f32", max_iter=50, flip_sets=hx4)
    e4 = (rng.random((96, hz4.shape[1])) < 0.01).astype(np.uint8)
    s4 = np.ascontiguousarray(((hz4 @ e4.T).T % 2).astype(np.uint8))
    a = dec4.decode(s4, want=("x", "iters", "status", "ssf_steps"))
    b = dec4.decode(pack_rows(s4), want=("x", "iters", "status", "ssf_steps"), packed=True)
    for k in a:
        assert np.array_equal(a[k], b[k]), ("c4", k)
