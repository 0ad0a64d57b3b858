"""Throughput benchmark: decoded syndrome shots/s + logical error rate on the
(3,4)-HGP n=225 code (BASELINE.json configs[1] = SURVEY §8(d) C2).

One step = one pass of the hot path over one batch per sweep point: for each
p in geomspace(1e-3, 1e-1, 9), decode B device-resident storage-experiment shots
(R = 0: H = Hz 108x225) with BP min-sum (max_iter 50, alpha_t = 1-2^-t)
+ small-set-flip on BP failures + fused logical-failure check.  Inputs for every
step are sampled on the device *before* the timed region (distinct shots per
step; on-device Philox sampler), so the timed region is decode only.

Precision: the headline line (`value`, `dtype`) runs BP in f64, ldpc v1's
message precision (its loops use double).  The same shots are then decoded in
f32 (the stated-tolerance variant) and reported under `variants`.

Output: rank 0 prints ONE JSON line of at most LINE_MAX_BYTES (the driver's
parser; round 5's 20 KB line was not read): the contract's fields, `roofline`,
`cpu_baseline`, the LER curve as one row of failures per p (the reference's own
record, misc/p_sweep.py:32-33) and one number + roofline fraction per extra
config (`configs`: C3, C4 f32 / f64, C5, the reference default).  The full
record (per-point roofline and LER, every config line, sub-records) goes to the
side file the line names (`detail`, --detail-out).

Inputs: the syndrome and readout rows are bit-packed u64 words by default
(QD_INPUT_PACKED: 48 B per shot at n = 225 instead of 333; the sampler writes
them, the triage reads them), --inputs bytes keeps one byte per bit.

Phases:
  1. headline: W warmup + K timed steps, the 9 points round-robin over --streams
     HIP streams (default 9: every point on its own stream; measured 79 vs 76 M
     f64 shots/s at 5), so kernels of independent points fill each other's tails;
     f64 wave kernels run at 12 waves per CU here (--wave-occupancy; a lone
     decode keeps 8, its own optimum); each point's steps run back to back on
     its stream and the streams join once, at the end of the timed region
     (--step-join end; joining them every step left each step's slowest point
     running alone at its end: 112.0 / 113.3 vs 116.9 / 117.3 M f64 shots/s,
     profiles/r05q/)
     (--schedule pipeline: every BP kernel on one stream and every SSF kernel on
     a second one behind an event -- measured slower: the persistent BP kernel
     fills every CU, so SSF only runs in BP's tail, which it cannot fill because
     it depends on that same BP kernel);
  2. f32 variant: the same shots, same timing protocol;
  3. isolated launches (--iso-steps, one stream): per-kernel durations from HIP
     events the library records on the launch stream around each kernel; the
     roofline uses these (overlapped launches share the chip, so their durations
     are not one kernel's);
  4. sampling + decode: K steps with the sampler inside the timed region;
  5. (rank 0, N = 1) `c3_line`: BASELINE config 3 ([[144,12,12]] BB lift,
     BP + SSF f64, 2^22 shots per p at p = 0.001 / 0.003 / 0.01);
     `large_code_roofline`: the HBM-bound path, BASELINE config 5 (n = 53,040
     Cayley-graph LP code, R = 1 spacetime syndromes) on the slot-group kernel,
     at two points where it decodes and the all-fail bandwidth point;
     `c4_line` (config 4's code, f64 and f32); `reference_default` (configs[0]'s
     bposd path with its compiled CPU leg).

Multi-GPU: `torchrun --nproc-per-node N bench.py --gpus N` (one process per
GPU), or `python bench.py --gpus N`, which starts that torchrun as a child
process before anything touches the GPU and exits with its status.  Shots are
sharded by index (rank r decodes shot range (step*N + r)*B ..), no data-path
collective; a barrier + synchronize brackets the timed region and rank 0
reports the max time over ranks.  value = shots decoded by all ranks / time.
The bookkeeping (barrier, max time, summed failure counts) runs on host words
over a gloo group (exp_ldpc_amd/sharding.py) on the GPU path and in the CPU
rehearsal alike; rank r uses HIP device r mod (visible devices), so N ranks
can also be rehearsed on one GPU.

Roofline (dominant kernel = the f64 BP kernel, named exactly as it ran by
Decoder.last_kernels()): its messages never leave the CU at n = 225, so
`bound` is "lds": `achieved` = algorithmic LDS bytes of the isolated launches
(32 B per edge + 16 B per check per BP iteration, times the launches' own
iteration totals) / their HIP-event durations, against the LDS's aggregate
peak.  The compulsory-HBM line (339 B of I/O per shot) sits beside it under
`roofline.hbm` and per sweep point under `roofline.per_point`; the PMC figures
of the same instantiation (profiles/*_pmc_summary.json; tools/pmc.sh +
tools/pmc_summary.py) give `ceilings` and `traffic` (HBM bytes per launch,
FETCH_SIZE x2 + WRITE_SIZE).
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from exp_ldpc_amd.sharding import barrier, gather_rows, max_time, reduce_counts  # noqa: E402  (pure Python, no GPU)

METRIC = "decoded syndrome shots/sec + logical error rate, (3,4)-HGP n=225 @ 1/2/4/8 GPUs"
CODE = "hgp_12_3_4_s1234"
SEED = 20250221
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
LDS_PEAK_GBS = 150000.0  # aggregate ds_read_b64/b128 rate, every CU streaming (MI355X_MICROARCH.md §LDS)
# per-CU LDS rates of the BP kernel's instructions (MI355X_MICROARCH.md §LDS table: B/clk/CU) and the
# clock the aggregate figures assume; stores move their data at a third of the read rate
LDS_CLK_GHZ, LDS_CUS = 2.4, 256
LDS_READ_B_PER_CLK, LDS_WRITE_B64_B_PER_CLK, LDS_WRITE_B128_B_PER_CLK = 256.0, 85.0, 79.0
OUT_BYTES_PER_SHOT = 1 + 1 + 4  # fail, status, iters out


def in_bytes_per_shot(m: int, n: int, packed: bool) -> int:
    """Input bytes the triage reads per shot: the syndrome and readout rows, as
    bytes (m + n) or as bit-packed u64 words (QD_INPUT_PACKED: 8 ceil(m/64) +
    8 ceil(n/64); 16 + 32 = 48 B at n = 225 instead of 333)."""
    return 8 * ((m + 63) // 64 + (n + 63) // 64) if packed else m + n


def wilson(k: int, n: int, z: float = 1.96):
    if n == 0:
        return (0.0, 1.0)
    ph = k / n
    den = 1 + z * z / n
    c = (ph + z * z / (2 * n)) / den
    h = z * math.sqrt(ph * (1 - ph) / n + z * z / (4 * n * n)) / den
    return (max(0.0, c - h), min(1.0, c + h))


def overlap(a, b) -> bool:
    return a[0] <= b[1] and b[0] <= a[1]


def load_code():
    from exp_ldpc_amd.codes import read_quantum_code
    with open(os.path.join(REPO, "tests", "golden", f"{CODE}.qecc")) as f:
        return read_quantum_code(f, validate_stabilizer_code=True)


def pmc_ceilings(kernel: str, **meta):
    """Per-launch PMC figures of exactly `kernel` (rocprof's spelling with its
    template arguments, as Decoder.last_kernels() reports it) from the newest
    committed PMC summary that holds it (profiles/*_pmc_summary.json, written by
    tools/pmc_summary.py from rocprofv3 --pmc passes of this bench command, or of
    one launch shape of it tagged by `meta`, e.g. c5_p=0.005), or None."""
    if not kernel:
        return None
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_summary.json")))
    for f in reversed(files):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except Exception:
            continue
        fm = d.get("meta", {})
        if any(fm.get(key) != val for key, val in meta.items()):
            continue
        for name, k in d.get("kernels", {}).items():
            if name.split("(", 1)[0] == kernel and "derived" in k:
                return os.path.relpath(f, REPO), name, k
    return None


def lds_roofline(bp_ms, pre_ms, listed, it_iso, args, hz, bp_kernel, ssf_kernel, ssf_ms):
    """Roofline of the dominant kernel, the BP kernel at n = 225: its messages
    never leave the CU, so the unit that bounds it is the LDS.  achieved =
    algorithmic LDS bytes of the isolated launches (per shot-iteration: every
    edge's v2c message read by its check (8 B) and written back by its variable
    (8 B), every edge's (m1, m2) check state gathered by its variable (16 B),
    every check's state written (16 B)) / the BP kernel's own HIP-event
    duration.  Only the shots the BP kernel decoded count: on the two-pass path
    the triage finishes zero-syndrome and iteration-1-converged shots itself
    (they report 1 iteration and never touch the BP kernel's LDS), so a launch's
    iterations are sum(iters) - (B - listed), listed = the triage's compact-list
    length; the triage's own time (HBM-streaming, `triage`) is kept out of the
    BP kernel's and reported beside it.  peak = the LDS's aggregate rate with
    every CU streaming (MI355X_MICROARCH.md §LDS: ~150 TB/s for
    ds_read_b64/b128).  The HBM line (compulsory I/O per shot) is kept beside it,
    per launch and per sweep point."""
    E, m = int(hz.nnz), int(hz.shape[0])
    lds_per_it = 32 * E + 16 * m
    tri_shot = in_bytes_per_shot(m, int(hz.shape[1]), args.inputs == "packed")
    io_shot = tri_shot + OUT_BYTES_PER_SHOT
    B = args.batch
    it_bp = np.where(listed >= 0, it_iso - (B - listed), it_iso).astype(np.float64)
    stage_ms = bp_ms + pre_ms
    tot_ms = float(bp_ms.sum())
    lds_bytes = float(lds_per_it * it_bp.sum())
    achieved = lds_bytes / (tot_ms * 1e-3) / 1e9
    io_launch = io_shot * B
    hbm_ach = io_launch / (stage_ms.mean() * 1e-3) / 1e9
    tri_bytes = tri_shot * B
    per_point = {}
    for pi in range(bp_ms.shape[1]):
        ms = float(bp_ms[:, pi].mean())
        st = float(stage_ms[:, pi].mean())
        tr = float(pre_ms[:, pi].mean())
        per_point[str(pi)] = {"bp_ms": ms, "triage_ms": tr, "bp_stage_ms": st,
                              "listed_frac": float(listed[:, pi].mean() / B) if (listed[:, pi] >= 0).all() else None,
                              "hbm_frac": io_launch / (st * 1e-3) / 1e9 / HBM_PEAK_GBS,
                              "lds_frac": lds_per_it * float(it_bp[:, pi].mean()) / (ms * 1e-3) / 1e9 / LDS_PEAK_GBS,
                              "triage_hbm_frac": tri_bytes / (tr * 1e-3) / 1e9 / HBM_PEAK_GBS if tr > 0 else None}
    # the same bytes against the LDS time floor of their instruction mix: reads
    # (rows 8 B/edge, state gathers 16 B/edge) at the read rate, the v2c scatter
    # (ds_write_b64, 8 B/edge) and the state writes (ds_write_b128, 16 B/check)
    # at their store rates
    agg = LDS_CUS * LDS_CLK_GHZ  # G clk/s over the chip
    t_floor = (24 * E / (LDS_READ_B_PER_CLK * agg) + 8 * E / (LDS_WRITE_B64_B_PER_CLK * agg) +
               16 * m / (LDS_WRITE_B128_B_PER_CLK * agg))  # ns per shot-iteration
    mix_peak = lds_per_it / t_floor  # GB/s
    return {"bound": "lds", "achieved": achieved, "peak": LDS_PEAK_GBS, "unit": "GB/s", "frac": achieved / LDS_PEAK_GBS,
            "mix": {"peak": mix_peak, "frac": achieved / mix_peak,
                    "model": f"LDS time floor of the kernel's instruction mix: {24 * E} B of reads at "
                             f"{LDS_READ_B_PER_CLK:.0f} B/clk/CU, {8 * E} B of ds_write_b64 at "
                             f"{LDS_WRITE_B64_B_PER_CLK:.0f}, {16 * m} B of ds_write_b128 at "
                             f"{LDS_WRITE_B128_B_PER_CLK:.0f} (MI355X_MICROARCH.md LDS table), {LDS_CUS} CUs at "
                             f"{LDS_CLK_GHZ} GHz: {t_floor * 1e3:.0f} ps per shot-iteration"},
            "traffic": None, "kernel": bp_kernel, "avg_launch_ms": float(bp_ms.mean()), "launches": int(bp_ms.size),
            "timing": "HIP events recorded by the library on the launch stream around the BP kernel alone (the "
                      "triage pass before it has its own event pair), isolated phase (one stream)",
            "algorithmic_bytes_per_launch": lds_bytes / bp_ms.size,
            "bytes_model": f"LDS: 32 B per edge + 16 B per check per BP iteration ({lds_per_it} B per shot-iteration "
                           f"at E={E}, m={m}) x the iterations of the shots the BP kernel decoded "
                           "(sum(iters) - (B - listed))",
            "hbm": {"achieved": hbm_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_ach / HBM_PEAK_GBS,
                    "algorithmic_bytes_per_launch": io_launch,
                    "bytes_model": f"per shot {io_shot} B compulsory HBM I/O ({tri_shot} B of syndrome + "
                                   f"readout rows in ({args.inputs}), fail + status + int32 iterations out) over "
                                   "the BP stage (triage + BP kernel)"},
            "triage": {"avg_launch_ms": float(pre_ms.mean()),
                       "achieved": tri_bytes / (float(pre_ms.mean()) * 1e-3) / 1e9 if pre_ms.mean() > 0 else None,
                       "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "bytes_model": f"{tri_shot} B per shot: syndrome + readout rows ({args.inputs}) read once"},
            "per_point": per_point,
            "ssf_kernel": ssf_kernel, "ssf_avg_launch_ms": float(ssf_ms.mean()),
            "isolated_step_ms": float(stage_ms.sum(axis=1).mean() + ssf_ms.sum(axis=1).mean())}


def launch_children(args) -> int:
    """`python bench.py --gpus N` without a launcher: run torchrun with N ranks as
    a child process (nothing here has touched the GPU) and return its status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _cpu_leg(orc, code, ps, per_p, precision, threads):
    """Decode per_p oracle-sampled shots at every point in `precision`; returns
    (seconds of decode, failures per point)."""
    hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
    elapsed = 0.0
    fails = {}
    for pi, p in enumerate(ps):
        syn, rd = orc.sample_storage(hz, 0, p, p, seed=SEED, stream=pi, shot0=0, B=per_p, nthreads=threads)
        t0 = time.perf_counter()
        out = orc.decode(hz, 2 * p / 3, syn, method="ms", precision=precision, max_iter=50, ssf=True, gens=hx, lz=lz,
                         readout=rd, want_llr=False, nthreads=threads, ssf_impl="fast")
        elapsed += time.perf_counter() - t0
        fails[f"{p:.6g}"] = int(out["fail"].sum())
    return elapsed, fails


def cpu_baseline(code, ps, args):
    """Time the CPU oracle (C port of the same algorithm, OpenMP over shots) on a
    bounded sample of the same workload: f64 like ldpc (the baseline `value`;
    its failure counts give the CPU LER curve the GPU curves are compared with)
    and f32 beside it (`variants`, the same-precision figure for the GPU's f32
    variant line)."""
    from oracle import load as load_oracle
    orc = load_oracle()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    per_p = args.cpu_shots
    elapsed, fails = _cpu_leg(orc, code, ps, per_p, "f64", threads)
    total = per_p * len(ps)
    res = {"value": total / elapsed, "unit": "shots/s", "cores": threads, "kind": "port", "dtype": "f64",
           "sample": f"{per_p} shots at each of the {len(ps)} sweep points (same sampler and seed as the GPU run, "
                     f"shot indices 0..{per_p - 1}, i.e. the warmup step's shots, disjoint from the timed ones); "
                     f"BP min-sum f64 max_iter 50 + SSF + logical check, decode only; {elapsed:.1f} s of CPU work "
                     f"on {threads} threads",
           "failures_per_point": fails, "shots_per_point": per_p}
    per32 = max(1, per_p // 2)
    if args.variant == "f32" or args.precision == "f32":
        e32, f32 = _cpu_leg(orc, code, ps, per32, "f32", threads)
        res["variants"] = [{"dtype": "f32", "value": per32 * len(ps) / e32, "unit": "shots/s", "cores": threads,
                            "sample": f"{per32} shots per point (shot indices 0..{per32 - 1}), BP min-sum f32, "
                                      f"otherwise as the f64 leg; {e32:.1f} s of CPU work",
                            "failures_per_point": f32, "shots_per_point": per32}]
    return res


def large_code_roofline(dev, shots: int = 1 << 16, ps=(0.0005, 0.001, 0.005), warm_shots: int = 1 << 13,
                        low_p_shots: int = 1 << 18):
    """HBM roofline of the genuinely HBM-bound path: BASELINE config 5 (PSL(2,16)
    Cayley-graph LP code, n = 53,040) at R = 1 spacetime syndromes (H_st
    48,960 x 130,560, E = 236,640), BP min-sum f64 max_iter 50 + fold + logical
    check on the slot-group kernel, whose messages stream through HBM.  Per p:
    one warmup launch, one timed launch (HIP events around the BP kernel on its
    launch stream).  The low points (p = 0.0005, 0.001) are where BP converges
    at R = 1 and the code decodes (k = 4080 logicals: at p = 0.002 the LER is
    already 0.74, profiles/r06a); the last (0.005) is the worst case where
    every shot runs all 50 iterations (LER ~1), kept as the bandwidth figure.
    The warmup launch decodes 2^13 shots (module load, scratch sizing;
    tools/gpu/lines_only.py --c5-warm-full makes it the timed launch's twin, so
    a PMC pass's per-dispatch average is that launch's).  The decoding points
    (p <= 0.001) decode `low_p_shots` = 2^18 shots per launch: the slot-group
    kernel keeps ~32 k slots in flight, and with 2^16 shots (two per slot) a
    group streamed its finished slots' lines through a long tail (PMC 1.22x the
    algorithmic bytes at p = 0.001, profiles/r06_c5_p001_pmc_summary.json);
    the all-fail point keeps 2^16 (every shot runs 50 iterations, no tail).
    Algorithmic bytes = 32 B per edge per shot-iteration (f64 v2c read + c2v
    write in the check pass, c2v read + v2c write in the column pass) + the
    per-shot I/O (syndrome, readout, outputs)."""
    import scipy.sparse as sp
    import torch
    from exp_ldpc_amd.decoder import Decoder
    from exp_ldpc_amd.spacetime import SpacetimeCode

    def csr(path, key):  # committed fixture (tools/fixtures/make_c5_fixture.py)
        d = np.load(os.path.join(REPO, "tests", "golden", path))
        return sp.csr_matrix((np.ones(d[key + "_indices"].size, np.uint8), d[key + "_indices"], d[key + "_indptr"]),
                             shape=tuple(d[key + "_shape"]))
    hz = csr("lp_pgl2_1_4_2_s1_checks.npz", "hz")
    lz = csr("lp_pgl2_1_4_2_s1_logicals.npz", "lz")
    H = sp.csr_matrix(SpacetimeCode(hz, 1).spacetime_check_matrix)
    m, n = H.shape
    nd = hz.shape[1]
    E = int(H.nnz)
    sampler = Decoder(hz, 2 * ps[0] / 3, method="ms", precision="f64", max_iter=50, device=dev.index)
    dec = Decoder(H, 2 * ps[0] / 3, method="ms", precision="f64", max_iter=50, logicals=lz, n_data=nd, fold_blocks=2,
                  device=dev.index)
    top = max([shots] + [low_p_shots for p in ps if p <= 0.001])
    wmax = min(top, warm_shots)
    # warmup rows [0, wmax), timed rows [wmax, wmax + top)
    syn = torch.empty((wmax + top, m), dtype=torch.uint8, device=dev)
    rd = torch.empty((wmax + top, nd), dtype=torch.uint8, device=dev)
    iters = torch.empty(wmax + top, dtype=torch.int32, device=dev)
    status = torch.empty(wmax + top, dtype=torch.uint8, device=dev)
    fail = torch.empty(wmax + top, dtype=torch.uint8, device=dev)
    kernel = "qdec::bp_group_kernel<double, 1, 8, 4>"
    lines = []
    full = shots
    for p in ps:
        shots = low_p_shots if p <= 0.001 else full
        warm = min(shots, warm_shots)
        dec.set_priors(np.full(n, 2 * p / 3))
        sampler.sample_storage_device(1, p, p, SEED, 100, 0, warm, syn[:warm], rd[:warm])
        sampler.sample_storage_device(1, p, p, SEED, 100, top, shots, syn[wmax:wmax + shots], rd[wmax:wmax + shots])
        dec.decode_device(warm, syn=syn[:warm], readout=rd[:warm], iters=iters[:warm], status=status[:warm],
                          fail=fail[:warm])
        torch.cuda.synchronize(dev)
        dec.set_timing(1)
        t0 = time.perf_counter()
        T = slice(wmax, wmax + shots)
        dec.decode_device(shots, syn=syn[T], readout=rd[T], iters=iters[T], status=status[T], fail=fail[T])
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        bp_ms, _ = dec.read_timing()
        kernel = dec.last_kernels()[0] or kernel
        it_sum = int(iters[T].to(torch.int64).sum().item())
        io = shots * (m + nd + 1 + 1 + 4)
        algo = 32 * E * it_sum + io
        achieved = algo / (float(bp_ms[0]) * 1e-3) / 1e9
        row = {"p": p, "shots": shots, "shots_per_s": shots / wall, "bp_kernel_ms": float(bp_ms[0]),
               "mean_bp_iters": it_sum / shots,
               "bp_converged_frac": float((status[T] & 1).to(torch.float64).mean().item()),
               "ler": float(fail[T].to(torch.float64).mean().item()),
               "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": achieved / HBM_PEAK_GBS, "traffic": None, "algorithmic_bytes_per_launch": algo}}
        pmc = pmc_ceilings(kernel, c5_p=p, c5_shots=shots)  # PMC passes of exactly this launch shape
        if pmc is not None:
            src, name, k = pmc
            row["roofline"]["traffic"] = k["derived"].get("hbm_bytes_per_dispatch")
            row["roofline"]["traffic_source"] = src
            row["roofline"]["hbm_frac_pmc"] = k["derived"].get("hbm_frac")
        lines.append(row)
    res = {"config": "C5 as named: PSL(2,16) Cayley-graph LP (lifted_product_code_pgl2(1,4,2,double_cover=False,"
                     "seed=1)), n=53040 k=4080, R=1 spacetime 48960x130560 E=236640, BP min-sum f64 max_iter 50, "
                     f"fold + logical check, device-sampled, {low_p_shots} shots per launch at p <= 0.001, "
                     f"{full} above",
           "kernel": kernel,
           "bytes_model": "32 B per edge per shot-iteration (f64 messages: v2c read + c2v write, c2v read + v2c "
                          "write) + per-shot I/O",
           "lines": lines}
    del syn, rd, dec, sampler
    torch.cuda.empty_cache()
    return res


def c3_line(dev, shots: int = 1 << 22, ps=(0.001, 0.003, 0.01), precision: str = "f64", packed: bool = True):
    """BASELINE config 3 on one GPU: the [[144,12,12]] bivariate-bicycle lift
    (quasi-cyclic lifted product over Z_12 x Z_6, built by
    exp_ldpc_amd.lifted.bivariate_bicycle_code; reference construction
    matrix_lifted_product_code.py:105-212), R = 0 (Hz 72 x 144, E = 432), BP
    min-sum f64 max_iter 50 + SSF (Hx flip sets) + logical check.  Per p: one
    warmup launch and one timed launch of `shots` device-sampled shots (2^22:
    0.42 of the config's 1e7 per point), HIP events around the triage, BP and
    SSF kernels.  The BP kernel is the headline's wave kernel family, so the
    roofline is the headline's LDS model (32 B per edge + 16 B per check per
    shot-iteration of the shots the BP kernel decoded)."""
    import torch
    from exp_ldpc_amd.decoder import Decoder
    from exp_ldpc_amd.lifted import bivariate_bicycle_code
    code = bivariate_bicycle_code(12, 6, [(3, 0), (0, 1), (0, 2)], [(0, 3), (1, 0), (2, 0)], compute_logicals=True)
    hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
    m, n = hz.shape
    E = int(hz.nnz)
    lds_per_it = 32 * E + 16 * m
    if packed:
        syn = torch.empty((2, shots, (m + 63) // 64), dtype=torch.int64, device=dev)
        rd = torch.empty((2, shots, (n + 63) // 64), dtype=torch.int64, device=dev)
    else:
        syn = torch.empty((2, shots, m), dtype=torch.uint8, device=dev)
        rd = torch.empty((2, shots, n), dtype=torch.uint8, device=dev)
    iters = torch.empty((2, shots), dtype=torch.int32, device=dev)
    status = torch.empty((2, shots), dtype=torch.uint8, device=dev)
    fail = torch.empty((2, shots), dtype=torch.uint8, device=dev)
    steps = torch.empty((2, shots), dtype=torch.int32, device=dev)
    lines = []
    for p in ps:
        dec = Decoder(hz, 2 * p / 3, method="ms", precision=precision, max_iter=50, ms_scaling=0.0, flip_sets=hx,
                      logicals=lz, device=dev.index)
        for b in range(2):
            dec.sample_storage_device(0, p, p, SEED, 400, b * shots, shots, syn[b], rd[b], packed=packed)
        dec.decode_device(shots, syn=syn[0], readout=rd[0], iters=iters[0], status=status[0], fail=fail[0],
                          ssf_steps=steps[0], packed=packed)
        torch.cuda.synchronize(dev)
        dec.set_timing(1)
        t0 = time.perf_counter()
        dec.decode_device(shots, syn=syn[1], readout=rd[1], iters=iters[1], status=status[1], fail=fail[1],
                          ssf_steps=steps[1], packed=packed)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        pre_ms, bp_ms, ssf_ms, listed = dec.read_timing_detail()
        kern = dec.last_kernels()
        it_sum = int(iters[1].to(torch.int64).sum().item())
        it_bp = it_sum - (shots - int(listed[0])) if listed[0] >= 0 else it_sum
        ach = lds_per_it * it_bp / (float(bp_ms[0]) * 1e-3) / 1e9
        fails = int(fail[1].to(torch.int64).sum().item())
        lines.append({"p": p, "shots": shots, "shots_per_s": shots / wall, "failures": fails, "ler": fails / shots,
                      "wilson95": list(wilson(fails, shots)),
                      "bp_converged_frac": float((status[1] & 1).to(torch.float64).mean().item()),
                      "mean_bp_iters": it_sum / shots, "triage_ms": float(pre_ms[0]), "bp_kernel_ms": float(bp_ms[0]),
                      "ssf_kernel_ms": float(ssf_ms[0]), "listed_frac": float(listed[0]) / shots,
                      "bp_kernel": kern[0], "ssf_kernel": kern[1], "pre_kernel": kern[2],
                      "roofline": {"bound": "lds", "achieved": ach, "peak": LDS_PEAK_GBS, "unit": "GB/s",
                                   "frac": ach / LDS_PEAK_GBS, "traffic": None,
                                   "algorithmic_bytes_per_launch": lds_per_it * it_bp},
                      "hbm_frac_bp_stage": shots * (in_bytes_per_shot(m, n, packed) + OUT_BYTES_PER_SHOT)
                      / ((float(pre_ms[0]) + float(bp_ms[0])) * 1e-3) / 1e9 / HBM_PEAK_GBS})
        del dec
    del syn, rd
    torch.cuda.empty_cache()
    return {"config": f"C3: [[144,12,12]] bivariate-bicycle lift (BB 12x6, a=x^3+y+y^2, b=y^3+x+x^2), R=0 "
                      f"(Hz {m}x{n}, E={E}), BP min-sum {precision} max_iter 50 + SSF + logical check, {shots} "
                      "device-sampled shots per timed launch",
            "m": m, "n": n, "E": E, "bytes_model": f"LDS: 32 B per edge + 16 B per check per shot-iteration "
                                                   f"({lds_per_it} B) of the BP kernel's shots",
            "lines": lines}


def c4_line(dev, shots: int = 1 << 19, ps=(0.005, 0.01, 0.03), precisions=("f64", "f32")):
    """BASELINE config 4's code on one GPU (the driver's record of it; the
    config itself shards 1e7 shots over 8 GPUs exactly as the headline does):
    biregular_hgp(80, 3, 4, seed=2025), n = 10^4 (reference-generated checks,
    tests/golden/hgp_80_3_4_s2025_checks.npz; logicals fixture from
    tools/fixtures/make_c4_logicals.py), R = 0, BP min-sum max_iter 50 + SSF +
    logical check.  Per (precision, p): one warmup launch and one timed launch
    of `shots` device-sampled shots (2^19 at p <= 0.01, 2^18 at higher p),
    HIP events around the BP and SSF kernels.  The batch is large because the
    slot-group kernel's launch ends with each group's last shots: a group keeps
    streaming all 64 slots' lines while its slowest shot (up to 50 iterations)
    finishes, and at low p (2-6 iterations per shot) that tail weighs against
    2^17 / 256 groups = 512 shots per group; the config itself decodes 1e7
    shots.
    f64 runs bp_ms_lds64_kernel (v2c messages in registers, check states built
    by LDS atomics in one pass: LDS roofline, 44 B per edge + 16 B per check per
    shot-iteration; the slot-group kernel's HBM model, 32 B per edge per
    shot-iteration + I/O, applies when a handle forces it); f32 runs the LDS-resident kernel
    (every message on chip: LDS roofline, per shot-iteration 8 B per edge -- the
    variable pass reads the edge's c2v slot and writes its v2c back -- and 64 B
    per check -- the check pass reads its 32-B row of v2c and writes it back as
    c2v)."""
    import scipy.sparse as sp
    import torch
    from exp_ldpc_amd.decoder import Decoder

    def csr(path, key):
        d = np.load(os.path.join(REPO, "tests", "golden", path))
        return sp.csr_matrix((np.ones(d[key + "_indices"].size, np.uint8), d[key + "_indices"], d[key + "_indptr"]),
                             shape=tuple(d[key + "_shape"]))
    hz, hx = csr("hgp_80_3_4_s2025_checks.npz", "hz"), csr("hgp_80_3_4_s2025_checks.npz", "hx")
    lz = csr("hgp_80_3_4_s2025_logicals.npz", "lz")
    m, n = hz.shape
    E = int(hz.nnz)
    lines = []
    full = shots
    for p in ps:
        shots = full if p <= 0.01 else full // 2
        sampler = Decoder(hz, 2 * p / 3, method="ms", precision="f32", max_iter=50, device=dev.index)
        syn = torch.empty((2, shots, m), dtype=torch.uint8, device=dev)
        rd = torch.empty((2, shots, n), dtype=torch.uint8, device=dev)
        for b in range(2):
            sampler.sample_storage_device(0, p, p, SEED, 200, b * shots, shots, syn[b], rd[b])
        for prec in precisions:
            dec = Decoder(hz, 2 * p / 3, method="ms", precision=prec, max_iter=50, flip_sets=hx, logicals=lz,
                          device=dev.index)
            iters = torch.empty((2, shots), dtype=torch.int32, device=dev)
            status = torch.empty((2, shots), dtype=torch.uint8, device=dev)
            fail = torch.empty((2, shots), dtype=torch.uint8, device=dev)
            steps = torch.empty((2, shots), dtype=torch.int32, device=dev)
            dec.decode_device(shots, syn=syn[0], readout=rd[0], iters=iters[0], status=status[0], fail=fail[0],
                              ssf_steps=steps[0])
            torch.cuda.synchronize(dev)
            dec.set_timing(1)
            t0 = time.perf_counter()
            dec.decode_device(shots, syn=syn[1], readout=rd[1], iters=iters[1], status=status[1], fail=fail[1],
                              ssf_steps=steps[1])
            torch.cuda.synchronize(dev)
            wall = time.perf_counter() - t0
            bp_ms, ssf_ms = dec.read_timing()
            kern = dec.last_kernels()
            it_sum = int(iters[1].to(torch.int64).sum().item())
            io = shots * (m + n + 1 + 1 + 4)
            if "lds64" in kern[0]:
                algo = (44 * E + 16 * m) * it_sum
                roof = {"bound": "lds", "peak": LDS_PEAK_GBS,
                        "bytes_model": "LDS: 44 B per edge + 16 B per check per shot-iteration (one pass: 16-B "
                                       "(m1, m2) state + parity word read, ds_min_rtn_u64 on the next m1 (8 B out, "
                                       "8 B back), ds_min_u64 on its m2; check state reset), the data-dependent "
                                       "sign / decision xors not counted"}
            elif "group" in kern[0]:
                algo = 32 * E * it_sum + io
                roof = {"bound": "hbm", "peak": HBM_PEAK_GBS,
                        "bytes_model": "32 B per edge per shot-iteration (f64 messages through HBM: v2c read + c2v "
                                       "write, c2v read + v2c write) + per-shot I/O"}
            else:
                algo = (8 * E + 64 * m) * it_sum
                roof = {"bound": "lds", "peak": LDS_PEAK_GBS,
                        "bytes_model": "LDS: 8 B per edge + 64 B per check per shot-iteration (variable pass: c2v "
                                       "slot read + v2c write; check pass: 32-B row read + c2v row write)"}
            ach = algo / (float(bp_ms[0]) * 1e-3) / 1e9
            roof.update({"achieved": ach, "unit": "GB/s", "frac": ach / roof["peak"], "algorithmic_bytes_per_launch": algo,
                         "traffic": None})
            lines.append({"precision": prec, "p": p, "shots": shots, "shots_per_s": shots / wall,
                          "bp_kernel": kern[0], "ssf_kernel": kern[1], "bp_kernel_ms": float(bp_ms[0]),
                          "ssf_kernel_ms": float(ssf_ms[0]), "mean_bp_iters": it_sum / shots,
                          "bp_converged_frac": float((status[1] & 1).to(torch.float64).mean().item()),
                          "ler": float(fail[1].to(torch.float64).mean().item()), "roofline": roof})
            del dec
        del syn, rd, sampler
        torch.cuda.empty_cache()
    return {"config": "C4: biregular_hgp(80,3,4,seed=2025), n=10000 (BASELINE configs[3]'s code; 1 GPU, the "
                      "headline's shot sharding carries it to 8), R=0, BP min-sum max_iter 50 + SSF + logical check, "
                      f"{full} device-sampled shots per timed launch at p <= 0.01, {full // 2} above",
            "m": m, "n": n, "E": E, "lines": lines}


def reference_default_line(dev, code, shots: int = 1 << 18, batch: int = 1 << 16, p: float = 0.01,
                           cpu_shots: int = 1 << 16, cpu: bool = True):
    """The reference's own default decode (BASELINE configs[0]: scripts/p_sweep.py
    -> misc/p_sweep.py:57-78 defaults, _experiment.py:62-83,213-229): R = 1,
    decoder_mode bposd, product-sum BP, max_iter = n = 225, OSD-CS order 7,
    priors 2p/3, f64 BP (ldpc's message precision), through this package's
    p_sweep pipeline (BatchPipeline: BP kernel on H_st 216 x 558, OSD on the
    device for BP failures, fold + logical check).  GPU shots/s over `shots`
    device-sampled shots in `batch`-shot runs; BP time from the BP decoder's HIP
    events, OSD + the rest = the remainder.  CPU leg: the oracle's restatement of
    the same loop (oracle/harness_py.spacetime_bposd_corrections: the C ldpc-v1
    BP restatement + the C OSD restatement, both OpenMP over shots on the host's
    cores; a few OSD results re-checked against the numpy restatement, untimed)
    on the first `cpu_shots` of the same syndromes, BP and OSD timed apart,
    failure flags compared shot by shot."""
    import torch
    from exp_ldpc_amd.experiment import BatchPipeline
    from exp_ldpc_amd.noise_model import depolarizing_noise
    from exp_ldpc_amd.storage_sim import build_storage_simulation
    R = 1
    opts = {"max_iter": code.checks.num_qubits, "bp_method": "ps", "ms_scaling_factor": 0, "osd_method": "osd_cs",
            "osd_order": 7}
    priors = (2 * p / 3, 2 * p / 3)
    noise = depolarizing_noise(p, p)
    pipe = BatchPipeline(code, R, "bposd", opts, priors, noise=noise, precision="f64", device=dev.index)
    sim = build_storage_simulation(R, noise, code)
    nb = max(1, shots // batch)
    batches = [sim.sample_device(pipe.sampler_graph, batch, SEED, 300, b * batch) for b in range(nb)]
    first = pipe.run(*batches[0])  # warmup (also the shots the CPU leg decodes)
    torch.cuda.synchronize(dev)
    pipe.st.set_timing(nb)
    t0 = time.perf_counter()
    fails = conv = 0
    for syn, rd in batches:
        r = pipe.run(syn, rd)
        fails += int(r.fail.sum())
        conv += r.bp_converged
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    bp_ms, _ = pipe.st.read_timing()
    total = nb * batch
    res = {"config": "BASELINE configs[0] path (reference default): (3,4)-HGP n=225, R=1 (H_st 216x558), bposd, "
                     f"BP product-sum f64 max_iter {opts['max_iter']}, OSD-CS order 7, priors 2p/3, p={p}",
           "kernel": pipe.st.last_kernels()[0], "shots": total, "shots_per_s": total / wall,
           "ms_per_batch": wall / nb * 1e3, "batch": batch, "bp_ms_per_batch": float(bp_ms.mean()),
           "osd_and_rest_ms_per_batch": wall / nb * 1e3 - float(bp_ms.mean()),
           "bp_converged_frac": conv / total, "ler": fails / total}
    if cpu:
        from oracle import load as load_oracle
        from oracle.harness_py import _fold, _opts, _spacetime_matrix, logical_failures
        from oracle.osd_py import osd_decode
        orc = load_oracle()
        threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1), 64))
        syn_h = batches[0][0][:cpu_shots].cpu().numpy()
        rd_h = batches[0][1][:cpu_shots].cpu().numpy()
        Hst, prior = _spacetime_matrix(code.checks.z, R, *priors)
        kw = _opts(opts, "f64")
        t0 = time.perf_counter()
        out = orc.decode(Hst, prior, syn_h, method="ps", precision="f64", max_iter=kw["max_iter"], ms_scaling=0.0,
                         want_llr=True, nthreads=threads)
        t_bp = time.perf_counter() - t0
        x = out["x"].copy()
        bad = np.nonzero((out["status"] & 1) == 0)[0]
        t0 = time.perf_counter()
        if bad.size:  # compiled OSD-CS 7 (oracle/osd_impl.inc, OpenMP over the BP failures)
            x[bad] = orc.osd(Hst, syn_h[bad], out["llr"][bad], "osd_cs", 7, nthreads=threads)[1]
        t_osd = time.perf_counter() - t0
        # spot check of the compiled OSD against the numpy restatement (untimed)
        for b in bad[:8]:
            assert np.array_equal(x[b], osd_decode(Hst, syn_h[b], out["llr"][b], "osd_cs", 7)[1])
        corr = _fold(x, code.checks.z.shape[1], R)
        cpu_fail = logical_failures(code.logicals.z, rd_h, corr)
        res["cpu_baseline"] = {"value": cpu_shots / (t_bp + t_osd), "unit": "shots/s", "cores": threads, "kind": "port",
                               "sample": f"the first {cpu_shots} of the GPU run's shots; oracle BP (C, OpenMP) "
                                         f"{t_bp:.2f} s + compiled OSD-CS 7 (C, OpenMP) on {bad.size} BP failures "
                                         f"{t_osd:.3f} s",
                               "bp_s": t_bp, "osd_s": t_osd, "osd_impl": "C (oracle/osd_impl.inc), OpenMP",
                               "fail_flags_identical": bool(np.array_equal(cpu_fail, first.fail[:cpu_shots]))}
    del batches, pipe
    torch.cuda.empty_cache()
    return res


class FakeDecoder:
    """--fake-device (CPU tests of the launcher and the rank merge only): a
    stand-in with the decode_device signature; shot s fails iff (s + point) is odd."""

    def __init__(self, dev):
        self.dev = dev

    def sample_storage_device(self, rounds, p_data, p_meas, seed, stream_id, shot0, B, syn, readout, stream=None, **_):
        import torch
        syn.copy_(((torch.arange(shot0, shot0 + B, device=self.dev)[:, None] + stream_id) % 2).to(torch.uint8))
        readout.zero_()

    def decode_device(self, B, *, syn=None, readout=None, iters=None, status=None, fail=None, ssf_steps=None,
                      stream=None, **_):
        fail.copy_((syn[:, 0] == 1).to(fail.dtype))
        iters.fill_(1)
        status.fill_(3)
        ssf_steps.zero_()

    def set_timing(self, capacity):
        self.cap = capacity

    def set_wave_occupancy(self, waves_per_cu=0):
        pass

    def read_timing(self):
        return np.full(self.cap, 1e-3), np.full(self.cap, 1e-3)

    def read_timing_detail(self):
        return np.zeros(self.cap), np.full(self.cap, 1e-3), np.full(self.cap, 1e-3), np.full(self.cap, -1)


class Run:
    """Device-resident inputs and outputs of every step, and the timed loop."""

    def __init__(self, args, ps, m, n, world, rank, dev, torch, fake):
        self.args, self.ps, self.torch, self.dev = args, ps, torch, dev
        self.world, self.rank, self.fake = world, rank, fake
        self.B = args.batch
        self.nsteps = args.warmup + args.steps
        P = len(ps)
        u8 = dict(dtype=torch.uint8, device=dev)
        # inputs as byte rows or bit-packed u64 rows (--inputs; QD_INPUT_PACKED)
        self.packed = args.inputs == "packed"
        if self.packed:
            w = dict(dtype=torch.int64, device=dev)
            self.syn = torch.empty((self.nsteps, P, self.B, (m + 63) // 64), **w)
            self.rd = torch.empty((self.nsteps, P, self.B, (n + 63) // 64), **w)
        else:
            self.syn = torch.empty((self.nsteps, P, self.B, m), **u8)
            self.rd = torch.empty((self.nsteps, P, self.B, n), **u8)
        self.iters = torch.empty((self.nsteps, P, self.B), dtype=torch.int32, device=dev)
        self.status = torch.empty((self.nsteps, P, self.B), **u8)
        self.fail = torch.empty((self.nsteps, P, self.B), **u8)
        self.ssf_steps = torch.empty((self.nsteps, P, self.B), dtype=torch.int32, device=dev)
        self.ssf_stream = None
        self.ssf = False if args.no_ssf_exp else None  # None: the handle's flip sets decide (SSF on)
        if fake:
            self.streams = [None]
        else:
            main = torch.cuda.current_stream(dev)
            if args.stream_priority:
                # BP streams at the device's highest priority, SSF streams (below)
                # at the default: the dispatcher serves pending BP workgroups first
                hi = torch.cuda.Stream.priority_range()[1] if hasattr(torch.cuda.Stream, "priority_range") else -1
                self.streams = [torch.cuda.Stream(dev, priority=hi) for _ in range(max(1, args.streams))]
            else:
                self.streams = [main] + [torch.cuda.Stream(dev) for _ in range(max(1, args.streams) - 1)]
            if args.schedule == "pipeline":
                self.ssf_stream = torch.cuda.Stream(dev)
        # --ssf-streams: every point's SSF kernels on a stream of their own
        # (qd_graph_set_ssf_stream; the handle's two SSF queues let its next BP
        # stage run while this SSF kernel waits for a CU)
        self.ssf_streams = None
        if not fake and args.ssf_streams and args.schedule == "streams":
            self.ssf_streams = [torch.cuda.Stream(dev) for _ in ps]

    def shot0(self, s):
        return (s * self.world + self.rank) * self.B

    def sample(self, sampler, s, stream=None):
        for pi, p in enumerate(self.ps):
            sampler.sample_storage_device(0, p, p, SEED, pi, self.shot0(s), self.B, self.syn[s, pi], self.rd[s, pi],
                                          packed=self.packed, **({} if stream is None else {"stream": stream}))

    def sync(self):
        if not self.fake:
            self.torch.cuda.synchronize(self.dev)

    def barrier(self):
        barrier()  # sharding: CPU word over the gloo bookkeeping group

    def pipelined(self, decs, on: bool):
        """Route (or stop routing) the decoders' SSF kernels to the SSF stream(s)."""
        if self.fake:
            return
        if self.ssf_streams is not None:
            for d, st in zip(decs, self.ssf_streams):
                d.set_ssf_stream(st if on else None)
            return
        if self.ssf_stream is None:
            return
        for d in decs:
            d.set_ssf_stream(self.ssf_stream if on else None)

    def step(self, decs, s, streams):
        torch = self.torch
        if not self.fake and self.ssf_stream is not None and len(streams) > 1:
            # pipeline: BP kernels in point order on the main stream, each SSF on
            # the SSF stream behind its BP kernel; the main stream rejoins at the end
            for pi in range(len(self.ps)):
                decs[pi].decode_device(self.B, syn=self.syn[s, pi], readout=self.rd[s, pi], iters=self.iters[s, pi],
                                       status=self.status[s, pi], fail=self.fail[s, pi],
                                       ssf_steps=self.ssf_steps[s, pi], ssf=self.ssf, packed=self.packed, stream=streams[0].cuda_stream)
            ev = torch.cuda.Event()
            ev.record(self.ssf_stream)
            streams[0].wait_event(ev)
            return
        if self.fake or len(streams) == 1:
            for pi in range(len(self.ps)):
                decs[pi].decode_device(self.B, syn=self.syn[s, pi], readout=self.rd[s, pi], iters=self.iters[s, pi],
                                       status=self.status[s, pi], fail=self.fail[s, pi],
                                       ssf_steps=self.ssf_steps[s, pi], ssf=self.ssf, packed=self.packed,
                                       **({} if self.fake else {"stream": streams[0].cuda_stream}))
            return
        join = self.args.step_join == "step"
        if join:
            ev = torch.cuda.Event()
            ev.record(streams[0])
            for st in streams[1:]:
                st.wait_event(ev)
        order = range(len(self.ps)) if self.args.point_order == "asc" else range(len(self.ps) - 1, -1, -1)
        for j, pi in enumerate(order):
            st = streams[j % len(streams)]
            decs[pi].decode_device(self.B, syn=self.syn[s, pi], readout=self.rd[s, pi], iters=self.iters[s, pi],
                                   status=self.status[s, pi], fail=self.fail[s, pi], ssf_steps=self.ssf_steps[s, pi],
                                   ssf=self.ssf, packed=self.packed, stream=st.cuda_stream)
        if join:
            for st in streams[1:]:
                e2 = torch.cuda.Event()
                e2.record(st)
                streams[0].wait_event(e2)

    def timed(self, decs, steps, streams, sampler=None, warm=True):
        """Run the warmup steps (untimed, unless warm=False), then `steps` timed
        steps; returns the max-over-ranks wall time of the timed ones."""
        a = self.args
        for s in range(a.warmup if warm else 0):
            self.step(decs, s, streams)
        self.sync()
        self.barrier()
        self.sync()
        t0 = time.perf_counter()
        for s in range(a.warmup, a.warmup + steps):
            if sampler is not None:
                self.sample(sampler, s, None if self.fake else streams[0].cuda_stream)
            self.step(decs, s, streams)
        self.sync()
        self.barrier()
        self.local_elapsed = time.perf_counter() - t0  # this rank's own time (rank 0 reports every rank's)
        return max_time(self.local_elapsed)

    def counts(self):
        """Failures / BP-converged per point over the timed steps, summed over ranks."""
        torch = self.torch
        w = self.args.warmup
        fails = np.array(reduce_counts(self.fail[w:].to(torch.int64).sum(dim=(0, 2))))
        conv = np.array(reduce_counts((self.status[w:] & 1).to(torch.int64).sum(dim=(0, 2))))
        itp = self.iters[w:].to(torch.float64).mean(dim=(0, 2)).cpu().numpy()
        ssp = self.ssf_steps[w:].to(torch.float64).mean(dim=(0, 2)).cpu().numpy()
        return fails, conv, itp, ssp


LINE_MAX_BYTES = 8000  # the driver's parser; round 5's 20 KB line was not read (tests/test_bench_launcher.py)


def _r(x, nd: int = 4):
    """Round a float to `nd` significant digits for the compact line (None for
    a non-finite value: the line must stay strict JSON)."""
    if x is None or isinstance(x, (bool, int, str)):
        return x
    x = float(x)
    return float(f"{x:.{nd}g}") if math.isfinite(x) else None


def _finite(o):
    """Non-finite floats anywhere in a record -> None (strict JSON)."""
    if isinstance(o, float):
        return o if math.isfinite(o) else None
    if isinstance(o, dict):
        return {k: _finite(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_finite(v) for v in o]
    return o


def compact_line(full: dict, detail: str) -> dict:
    """The one stdout line rank 0 prints: the contract's fields, the roofline and
    CPU-baseline blocks, the LER curve as one row per p (the reference's own
    record, misc/p_sweep.py:32-33: p, failures, samples), and one number + its
    roofline fraction per extra config.  Everything else (per-point roofline,
    every config line, sub-records) stays in the side file `detail`."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data")
    line = {k: full[k] for k in keep if k in full}
    line["value"] = _r(line["value"], 6)
    line["ms_per_step"] = _r(line["ms_per_step"], 6)
    cfg = full["config"]
    line["config"] = {k: cfg[k] for k in ("workload", "shots_per_point_per_step_per_gpu", "global_batch", "parallelism",
                                          "inputs") if k in cfg}
    line["ranks_seen"] = full["ranks_seen"]
    line["ranks"] = [{"rank": x["rank"], "device": x["device"], "timed_s": _r(x["timed_s"], 6), "shots": x["shots"]}
                     for x in full["ranks"]][:16]
    rf = full["roofline"]
    roof = {k: _r(rf.get(k)) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "avg_launch_ms",
                                       "launches", "algorithmic_bytes_per_launch")}
    roof["kernel"] = rf.get("kernel")
    roof["bytes_model"] = "LDS: 32 B/edge + 16 B/check per shot-iteration of the BP kernel's shots"
    if "mix" in rf:  # the same bytes against the read+store time floor of the kernel's LDS instruction mix
        roof["mix"] = {"peak": _r(rf["mix"]["peak"]), "frac": _r(rf["mix"]["frac"])}
    if "lds_busy_pmc" in rf:
        roof["lds_busy_pmc"] = _r(rf["lds_busy_pmc"])
    if "ceilings" in rf:
        roof["lds_bank_conflict_ratio_pmc"] = _r(rf["ceilings"].get("lds_bank_conflict_ratio"))
        roof["pmc_source"] = rf["ceilings"].get("source")
    hb = rf.get("hbm", {})
    roof["hbm"] = {"achieved": _r(hb.get("achieved")), "frac": _r(hb.get("frac")), "peak": hb.get("peak")}
    tr = rf.get("triage", {})
    roof["triage"] = {"kernel": tr.get("kernel"), "avg_launch_ms": _r(tr.get("avg_launch_ms")),
                      "achieved": _r(tr.get("achieved")),
                      "frac": _r(tr["achieved"] / HBM_PEAK_GBS) if tr.get("achieved") else None}
    roof["ssf_kernel"] = rf.get("ssf_kernel")
    roof["ssf_avg_launch_ms"] = _r(rf.get("ssf_avg_launch_ms"))
    roof["isolated_step_ms"] = _r(rf.get("isolated_step_ms"))
    line["roofline"] = roof
    if "cpu_baseline" in full:
        cb = full["cpu_baseline"]
        line["cpu_baseline"] = {"value": _r(cb["value"]), "unit": cb["unit"], "cores": cb["cores"], "kind": cb["kind"],
                                "dtype": cb.get("dtype"), "sample": cb["sample"][:400]}
    if "ler_overlap_all" in full:
        line["ler_overlap_all"] = full["ler_overlap_all"]
    ler = full.get("ler", {})
    if ler:
        rows = list(ler.values())
        cur = {"p": [_r(float(k)) for k in ler], "shots": rows[0]["shots"], "failures": [r["failures"] for r in rows]}
        if "cpu_f64" in rows[0]:
            cur["cpu_f64_shots"] = rows[0]["cpu_f64"]["shots"]
            cur["cpu_f64_failures"] = [r["cpu_f64"]["failures"] for r in rows]
        for v in full.get("variants", []):
            if v["dtype"] in rows[0]:
                cur[v["dtype"] + "_failures"] = [r[v["dtype"]]["failures"] for r in rows]
        line["ler"] = cur
    if "variants" in full:
        line["variants"] = [{"dtype": v["dtype"], "value": _r(v["value"], 6), "ms_per_step": _r(v["ms_per_step"], 5)}
                            for v in full["variants"]]
    if "sample_and_decode" in full:
        line["sample_and_decode"] = _r(full["sample_and_decode"]["value"], 5)
    cfgs = {}
    if "c3_line" in full:
        ls = full["c3_line"]["lines"]
        cfgs["c3"] = {"dtype": "f64", "p": [x["p"] for x in ls], "shots_per_s": [_r(x["shots_per_s"]) for x in ls],
                      "frac": [_r(x["roofline"]["frac"], 3) for x in ls], "bound": "lds",
                      "ler": [_r(x["ler"], 3) for x in ls], "kernel": ls[0]["bp_kernel"] if ls else None}
    if "c4_line" in full:
        ls = full["c4_line"]["lines"]
        for prec in sorted({x["precision"] for x in ls}):
            sel = [x for x in ls if x["precision"] == prec]
            cfgs["c4_" + prec] = {"p": [x["p"] for x in sel], "shots_per_s": [_r(x["shots_per_s"]) for x in sel],
                                  "frac": [_r(x["roofline"]["frac"], 3) for x in sel],
                                  "bound": sel[0]["roofline"]["bound"], "kernel": sel[0]["bp_kernel"]}
    if "large_code_roofline" in full:
        lc = full["large_code_roofline"]
        ls = lc["lines"]
        cfgs["c5"] = {"dtype": "f64", "p": [x["p"] for x in ls], "shots_per_s": [_r(x["shots_per_s"]) for x in ls],
                      "frac": [_r(x["roofline"]["frac"], 3) for x in ls], "bound": "hbm",
                      "traffic": [_r(x["roofline"]["traffic"]) for x in ls], "ler": [_r(x["ler"], 3) for x in ls],
                      "kernel": lc["kernel"]}
    if "reference_default" in full:
        rd = full["reference_default"]
        cfgs["reference_default"] = {"shots_per_s": _r(rd["shots_per_s"]), "ler": _r(rd["ler"], 3),
                                     "kernel": rd["kernel"]}
        if "cpu_baseline" in rd:
            c = rd["cpu_baseline"]
            cfgs["reference_default"]["cpu"] = {"value": _r(c["value"]), "cores": c["cores"],
                                                "osd": c.get("osd_impl"),
                                                "fail_flags_identical": c["fail_flags_identical"]}
    if cfgs:
        line["configs"] = cfgs
    line["detail"] = detail
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1 << 18, help="shots per sweep point per step per GPU")
    ap.add_argument("--points", type=int, default=9)
    ap.add_argument("--p", type=float, action="append", help="decode only these p values (diagnostics)")
    ap.add_argument("--precision", default="f64", choices=["f32", "f64"], help="headline BP precision")
    ap.add_argument("--variant", default="f32", choices=["f32", "f64", "none"],
                    help="second precision decoded on the same shots (reported under variants)")
    ap.add_argument("--cpu-shots", type=int, default=200000, help="CPU-baseline shots per sweep point")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--streams", type=int, default=9, help="HIP streams the sweep points are spread over "
                                                           "(--schedule streams)")
    ap.add_argument("--schedule", default="streams", choices=["pipeline", "streams"],
                    help="pipeline: every BP kernel on one stream, every SSF kernel on a second one behind an "
                         "event (point i's SSF overlaps point i+1's BP); streams: points round-robin over "
                         "--streams streams")
    ap.add_argument("--wave-occupancy", type=int, default=-1,
                    help="waves per CU of the wave BP kernels in the overlapped phases (qd_graph_set_wave_occupancy); "
                         "-1 = 12 for f64 when the points share the chip over several streams, else the default")
    ap.add_argument("--step-join", default="end", choices=["step", "end"],
                    help="streams schedule: join every point's stream at the end of each step (step) or only at the "
                         "end of the timed region (end: each point's steps run back to back on its stream)")
    ap.add_argument("--point-order", default="asc", choices=["asc", "desc"],
                    help="launch order of the sweep points in the overlapped phases (desc: highest p first)")
    ap.add_argument("--iso-steps", type=int, default=2, help="isolated (one-stream) steps timing each kernel")
    ap.add_argument("--no-sample-phase", action="store_true", help="skip the sampling+decode phase")
    ap.add_argument("--no-large-code", action="store_true",
                    help="skip the config-5 HBM-roofline line (large_code_roofline; rank 0, N=1 only)")
    ap.add_argument("--no-c4", action="store_true", help="skip the config-4 code line (c4_line; rank 0, N=1 only)")
    ap.add_argument("--no-reference-default", action="store_true",
                    help="skip the reference-default bposd line (reference_default_line; rank 0, N=1 only)")
    ap.add_argument("--inputs", default="packed", choices=["packed", "bytes"],
                    help="device input rows: bit-packed u64 words (QD_INPUT_PACKED; the sampler writes them) or one "
                         "byte per bit")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="side file (relative to the repo root unless absolute) for the full record: per-point LER "
                         "and roofline, every config line; the stdout line names it")
    ap.add_argument("--no-c3", action="store_true", help="skip the config-3 line (c3_line; rank 0, N=1 only)")
    ap.add_argument("--fake-device", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--ssf-streams", type=int, default=1, choices=[0, 1],
                    help="streams schedule: 1 (default) = every point's SSF kernels on their own stream (split SSF, "
                         "double-buffered queues), 0 = on the point's stream behind its BP kernel")
    ap.add_argument("--ssf-fuse", type=int, default=0, choices=[0, 1],
                    help="1: SSF inside the compact BP kernel (QD_OPT_SSF_FUSE); 0: queue + ssf_lut_kernel")
    # diagnostic: decode without SSF (prices SSF inside the overlapped step)
    ap.add_argument("--no-ssf-exp", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--stream-priority", type=int, default=1, choices=[0, 1],
                    help="1 (default): the points' BP streams at the device's high priority, the SSF streams at "
                         "the default one (the dispatcher serves pending BP workgroups first: +2.5 %% against "
                         "equal priorities, profiles/r06p/); 0: equal priorities")
    args = ap.parse_args()
    args.iso_steps = max(1, min(args.iso_steps, args.steps))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_children(args))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    from exp_ldpc_amd.sharding import init_process_group, rank_device

    fake = args.fake_device
    if world > 1:  # the same gloo bookkeeping group on the GPU path and the CPU rehearsal
        init_process_group()
    if fake:
        dev = torch.device("cpu")
    else:
        local = rank_device(local, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)

    code = load_code()
    hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
    m, n = hz.shape
    ps = np.geomspace(1e-3, 1e-1, args.points) if not args.p else np.array(args.p)
    P = len(ps)

    def decoders(precision):
        if fake:
            return [FakeDecoder(dev) for _ in ps]
        from exp_ldpc_amd.decoder import Decoder
        # one decoder graph per sweep point (priors differ), sharing nothing mutable
        ds = [Decoder(hz, 2 * p / 3, method="ms", precision=precision, max_iter=50, ms_scaling=0.0,
                      flip_sets=hx, logicals=lz, device=local) for p in ps]
        for d in ds:
            d.set_option("ssf_fuse", args.ssf_fuse)
        return ds

    run = Run(args, ps, m, n, world, rank, dev, torch, fake)
    decs = decoders(args.precision)
    for s in range(run.nsteps):  # distinct shots for every (step, point), sampled on device
        run.sample(decs[0], s)
    run.sync()

    def occupancy(precision):
        """Waves per CU for the overlapped phases: concurrent points (several
        streams) run f64 at full occupancy, 12 waves per CU (82-83 vs 80 M
        shots/s at 8, profiles/r03_ab_layout/occupancy_streams_sweep.json); a
        lone decode keeps the default (8: faster alone)."""
        if args.wave_occupancy >= 0:
            return args.wave_occupancy
        return 12 if precision == "f64" and args.schedule == "streams" and len(run.streams) > 1 else 0

    def set_occupancy(dset, w):
        for d in dset:
            d.set_wave_occupancy(w)

    # ---- phase 1: headline precision, overlapped (pipeline or streams) ----
    occ = {args.precision: occupancy(args.precision)}
    set_occupancy(decs, occ[args.precision])
    run.pipelined(decs, True)
    elapsed = run.timed(decs, args.steps, run.streams)
    run.pipelined(decs, False)
    fails, conv, itp, ssp = run.counts()
    # per-rank record of the headline phase: a straggler, a shared device or a
    # missing rank is visible in rank 0's line
    rank_rows = gather_rows([rank, -1 if fake else dev.index, run.local_elapsed, args.steps * args.batch * len(ps)])
    shots_per_point = args.steps * args.batch * world
    total_shots = shots_per_point * P

    # ---- phase 2: the other precision on the same shots ----
    variant = None
    if args.variant not in ("none", args.precision):
        vdecs = decoders(args.variant)
        occ[args.variant] = occupancy(args.variant)
        set_occupancy(vdecs, occ[args.variant])
        run.pipelined(vdecs, True)
        v_elapsed = run.timed(vdecs, args.steps, run.streams)
        run.pipelined(vdecs, False)
        v_fails, v_conv, _, _ = run.counts()
        variant = (args.variant, v_elapsed, v_fails, v_conv, vdecs)

    # ---- phase 3: isolated launches (one stream) for per-kernel durations ----
    iso = {}
    for prec, dset in [(args.precision, decs)] + ([(variant[0], variant[4])] if variant else []):
        set_occupancy(dset, 0)  # one stream: the lone-decode default
        for d in dset:
            d.set_timing(args.iso_steps)
        run.timed(dset, args.iso_steps, run.streams[:1], warm=False)  # every launch is timed
        bp_ms = np.zeros((args.iso_steps, P))
        pre_ms = np.zeros((args.iso_steps, P))
        ssf_ms = np.zeros((args.iso_steps, P))
        listed = np.zeros((args.iso_steps, P), np.int64)
        for pi, d in enumerate(dset):
            t_pre, t_bp, t_ssf, n_list = d.read_timing_detail()
            pre_ms[:, pi] = t_pre[:args.iso_steps]
            bp_ms[:, pi] = t_bp[:args.iso_steps]
            ssf_ms[:, pi] = t_ssf[:args.iso_steps]
            listed[:, pi] = n_list[:args.iso_steps]
        it_iso = run.iters[args.warmup:args.warmup + args.iso_steps].to(torch.int64).sum(dim=2).cpu().numpy()
        names = ("", "", "") if fake else dset[-1].last_kernels()  # the instantiations the isolated phase ran
        iso[prec] = (bp_ms, ssf_ms, it_iso, names, pre_ms, listed)

    # ---- phase 4: sampling + decode in the timed region ----
    sd = None
    if not args.no_sample_phase:
        sd_elapsed = run.timed(decs, args.steps, run.streams[:1], sampler=decs[0], warm=False)
        sd = total_shots / sd_elapsed

    large = c4 = refdef = c3 = None
    if rank == 0 and world == 1 and not fake and not args.no_c3:
        c3 = c3_line(dev, packed=args.inputs == "packed")
    if rank == 0 and world == 1 and not fake and not args.no_large_code:
        large = large_code_roofline(dev)
    if rank == 0 and world == 1 and not fake and not args.no_c4:
        c4 = c4_line(dev)
    if rank == 0 and world == 1 and not fake and not args.no_reference_default:
        refdef = reference_default_line(dev, code, cpu=not args.no_cpu_baseline)

    if rank == 0:
        value = total_shots / elapsed
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(code, ps, args)
        ler = {}
        for pi, p in enumerate(ps):
            key = f"{p:.6g}"
            w_h = wilson(int(fails[pi]), shots_per_point)
            row = {"failures": int(fails[pi]), "shots": shots_per_point, "ler": float(fails[pi] / shots_per_point),
                   "wilson95": list(w_h), "bp_converged_frac": float(conv[pi] / shots_per_point),
                   "mean_bp_iters_rank0": float(itp[pi]), "mean_ssf_steps_rank0": float(ssp[pi]),
                   "bp_kernel_ms_isolated": float(iso[args.precision][0][:, pi].mean()),
                   "triage_ms_isolated": float(iso[args.precision][4][:, pi].mean()),
                   "ssf_kernel_ms_isolated": float(iso[args.precision][1][:, pi].mean())}
            cw = None
            if cpu is not None:
                cw = wilson(cpu["failures_per_point"][key], cpu["shots_per_point"])
                row["cpu_f64"] = {"failures": cpu["failures_per_point"][key], "shots": cpu["shots_per_point"],
                                  "wilson95": list(cw)}
                row["overlaps_cpu_f64"] = overlap(w_h, cw)
            if variant:
                vw = wilson(int(variant[2][pi]), shots_per_point)
                vr = {"failures": int(variant[2][pi]), "wilson95": list(vw),
                      "bp_converged_frac": float(variant[3][pi] / shots_per_point),
                      "overlaps_headline": overlap(vw, w_h)}
                if cw is not None:
                    vr["overlaps_cpu_f64"] = overlap(vw, cw)
                row[variant[0]] = vr
            ler[key] = row

        bp_ms, ssf_ms, it_iso, (bp_kernel, ssf_kernel, pre_kernel), pre_ms, listed = iso[args.precision]
        roof = lds_roofline(bp_ms, pre_ms, listed, it_iso, args, hz, bp_kernel, ssf_kernel, ssf_ms)
        if pre_kernel:
            roof["pre_kernel"] = pre_kernel
            roof["triage"]["kernel"] = pre_kernel
        pmc = None if fake else pmc_ceilings(bp_kernel)
        if pmc is not None:
            src, name, k = pmc
            dv = k["derived"]
            roof["traffic"] = dv.get("hbm_bytes_per_dispatch")
            roof["ceilings"] = {"source": src, "kernel": name,
                                **{key: dv.get(key) for key in ("valu_issue_frac", "lds_frac",
                                                                "lds_bank_conflict_ratio", "hbm_frac", "clock_ghz",
                                                                "duration_ms", "formulas")}}
            lf = dv.get("lds_frac")
            if lf is not None:
                roof["lds_busy_pmc"] = lf
        calib = os.path.join(REPO, "profiles", "r03_hbm_calibration")
        if os.path.isdir(calib):
            roof["hbm"]["traffic_calibration"] = {
                "source": os.path.relpath(calib, REPO),
                "note": "FETCH_SIZE of this kernel equals that of a staging-only build with the BP loop compiled "
                        "out (QDEC_CALIB_NOBP): the messages add no HBM bytes"}

        result = {
            "metric": METRIC, "value": value, "unit": "shots/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic: on-device Philox sampler of the storage experiment under depolarizing_noise(p, pm=p), "
                    "seed 20250221, distinct shots per step" + (" [FAKE DEVICE: launcher test]" if fake else ""),
            "config": {"workload": "C2: (3,4)-HGP n=225 (biregular_hgp(12,3,4,seed=1234)), R=0 (H=Hz 108x225, E=756), "
                                   f"p-sweep geomspace(1e-3,1e-1,9), BP min-sum {args.precision} max_iter=50 "
                                   "alpha_t=1-2^-t + SSF (Hx flip sets) + fused logical check",
                       "shots_per_point_per_step_per_gpu": args.batch, "global_batch": args.batch * P * world,
                       "parallelism": f"shot-sharded x{world}, no collective",
                       "inputs": "bit-packed u64 rows (QD_INPUT_PACKED)" if args.inputs == "packed" else "byte rows",
                       "schedule": args.schedule if args.schedule == "pipeline" else
                       f"{args.streams} streams, joined {'every step' if args.step_join == 'step' else 'at the end'}"
                       + (", SSF on a stream per point" if args.ssf_streams else "")
                       + (", BP streams at high priority" if args.stream_priority else ""),
                       "wave_waves_per_cu": {k: (v or "default") for k, v in occ.items()}},
        }
        if variant:
            vb, vs = iso[variant[0]][0], iso[variant[0]][1]
            result["variants"] = [{"dtype": variant[0], "value": total_shots / variant[1],
                                   "ms_per_step": variant[1] / args.steps * 1e3,
                                   "bp_kernel_ms_isolated_avg": float(vb.mean()),
                                   "ssf_kernel_ms_isolated_avg": float(vs.mean()),
                                   "note": "same shots, same protocol; LER per point under ler[p][dtype]"}]
        if sd is not None:
            result["sample_and_decode"] = {"value": sd, "unit": "shots/s", "dtype": args.precision, "streams": 1,
                                           "note": "on-device sampling inside the timed region, one stream"}
        result["ranks"] = [{"rank": int(r[0]), "device": int(r[1]), "timed_s": r[2], "shots": int(r[3]),
                            "shots_per_s": r[3] / r[2] if r[2] > 0 else None} for r in rank_rows]
        result["ranks_seen"] = len(rank_rows)
        result["roofline"] = roof
        if c3 is not None:
            result["c3_line"] = c3
        if large is not None:
            result["large_code_roofline"] = large
        if c4 is not None:
            result["c4_line"] = c4
        if refdef is not None:
            result["reference_default"] = refdef
        if cpu is not None:
            result["cpu_baseline"] = cpu
        result["ler"] = ler
        if cpu is not None:
            result["ler_overlap_all"] = {
                "headline_vs_cpu_f64": all(r["overlaps_cpu_f64"] for r in ler.values()),
                "variant_vs_cpu_f64": all(r[variant[0]]["overlaps_cpu_f64"] for r in ler.values()) if variant else None}
        detail = args.detail_out if os.path.isabs(args.detail_out) else os.path.join(REPO, args.detail_out)
        try:
            os.makedirs(os.path.dirname(detail), exist_ok=True)
            with open(detail, "w") as fh:
                json.dump(_finite(result), fh, indent=1, allow_nan=False)
        except OSError as e:  # the line still goes out; it says where the detail is not
            detail = f"unwritten ({e})"
        if os.path.isabs(detail) and detail.startswith(REPO + os.sep):
            detail = os.path.relpath(detail, REPO)
        print(json.dumps(_finite(compact_line(result, detail)), allow_nan=False))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
