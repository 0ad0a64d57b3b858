"""Batched storage-experiment harness: decoder modes, run_simulation, p_sweep.

Mirrors ``python/qldpc/misc/_experiment.py`` and ``python/qldpc/misc/p_sweep.py``
with the per-shot Python loop (``_experiment.py:200-209``) replaced by batched
device pipelines: shots are sampled on the GPU (storage_sim.StorageSim.
sample_device), decoded by libqdec_hip.so and reduced to failure counts on the
device.  Decoder modes (``--decoder_mode``):

  bposd              BP(+OSD) on the spacetime matrix, fold     (_experiment.py:62-83)
  bposd_hybrid       BP on spacetime, fold, then BP+OSD on H     (_experiment.py:85-126)
  bposd_single_shot  per-round [H|I] BP+OSD, then BP+OSD on H    (_experiment.py:12-60)
  bpssf              BP + small-set-flip on H (R = 0); R >= 1 runs bpssf_hybrid
  bpssf_hybrid       BP on spacetime, fold, then BP+SSF on H     (build-defined)
  bp                 BP only on the spacetime matrix
  bpd_detector       BP on the fault check matrix of a detector error model
                     (_experiment.py:128-151); the storage experiment's DEM is
                     written by dem.storage_experiment_dem (any R)

OSD runs on the GPU for the shots BP did not converge on (Decoder.osd_device,
csrc/qdec_osd.hip), fused with the fold and the failure check; graphs too large
for that kernel use the host stage (osd.py).
Logical failure = any(Lz (readout + correction)) mod 2 as at _experiment.py:209
(computed in-kernel for device stages).
"""
from __future__ import annotations

import math
import os
import re
import sys
import time
from argparse import ArgumentParser
from dataclasses import dataclass
from pathlib import Path
from typing import Callable, Dict, Tuple

import numpy as np
import scipy.sparse as sp

from . import _abi
from .codes import read_quantum_code
from .decoder import Decoder
from .osd import OsdSolver
from .spacetime import SpacetimeCode, SpacetimeCodeSingleShot
from .storage_sim import build_storage_simulation

__all__ = ["DECODER_MODES", "BatchPipeline", "ShardError", "run_shards", "BPOSDCorrect", "BPOSDHybridCorrect", "BPOSDCorrectSingleShot",
           "BPSSFCorrect", "BPDetectorCorrect", "run_simulation", "add_bposd_args", "unpack_bposd_args", "load_code", "p_sweep",
           "p_sweep_main", "parse_sweep_spec"]

DECODER_MODES = ["bposd", "bposd_single_shot", "bposd_hybrid", "bpd_detector", "bpssf", "bpssf_hybrid", "bp"]
DEFAULT_SEED = 20250221


def _torch():
    import torch
    return torch


@dataclass
class BatchResult:
    fail: np.ndarray          # bool[B]
    bp_converged: int
    iters_sum: int
    ssf_steps_sum: int
    corrections: np.ndarray | None = None  # uint8[B, n] when requested


class BatchPipeline:
    """One decoder mode on one device.  ``run(syn, readout)`` takes the sampler's
    device tensors (spacetime syndrome uint8[B,(R+1)m], readout uint8[B,n])."""

    def __init__(self, code, rounds: int, mode: str, bp_osd_options: Dict, priors: Tuple[float, float], *,
                 device: int = 0, precision: str = "f64", use_x_logicals: bool = False, osd_threads: int = 0,
                 noise=None):
        if mode not in DECODER_MODES:
            raise RuntimeError("Unknown decoder operation mode")
        if mode == "bpssf" and rounds > 0:
            mode = "bpssf_hybrid"
        self.mode = mode
        self.R = int(rounds)
        self.device = int(device)
        data_prior, meas_prior = priors
        H = code.checks.x if use_x_logicals else code.checks.z
        G = code.checks.z if use_x_logicals else code.checks.x
        L = code.logicals.x if use_x_logicals else code.logicals.z
        self.H = sp.csr_matrix(H)
        self.m, self.n = self.H.shape
        self.L = sp.csr_matrix(L) if sp.issparse(L) else np.asarray(L) % 2
        o = bp_osd_options
        common = dict(method=o.get("bp_method", "ps"), precision=precision, max_iter=int(o.get("max_iter", 0) or 0),
                      ms_scaling=float(o.get("ms_scaling_factor", 0.0)), device=self.device)
        osd_method = o.get("osd_method", "osd_cs")
        osd_order = int(o.get("osd_order", 0))
        self.osd_method, self.osd_order = osd_method, osd_order
        self.osd_threads = osd_threads
        R, n = self.R, self.n
        lz = self.L if self.L.shape[0] else None
        # spacetime stage (modes that use it)
        if mode in ("bposd", "bposd_hybrid", "bpssf_hybrid", "bp"):
            st = SpacetimeCode(self.H, R)
            Hst = st.spacetime_check_matrix
            prior = np.empty(Hst.shape[1])
            prior[st.true_data_slice()] = data_prior
            prior[(R + 1) * n:] = meas_prior
            self.st = Decoder(Hst, prior, n_data=n, fold_blocks=R + 1, logicals=lz, **common)
            self.st_osd = OsdSolver(Hst, osd_method, osd_order, osd_threads) if mode == "bposd" else None
        # final-round stage on H
        if mode in ("bposd_hybrid", "bposd_single_shot"):
            self.fin = Decoder(self.H, data_prior, logicals=lz, **common)
            self.fin_osd = OsdSolver(self.H, osd_method, osd_order, osd_threads)
        if mode in ("bpssf", "bpssf_hybrid"):
            self.fin = Decoder(self.H, data_prior, logicals=lz, flip_sets=G, ssf=True, **common)
        if mode == "bposd_single_shot":
            ss = SpacetimeCodeSingleShot(self.H)
            Hss = ss.spacetime_check_matrix
            prior = np.empty(Hss.shape[1])
            prior[:n] = data_prior
            prior[n:] = meas_prior
            self.ss = Decoder(Hss, prior, n_data=n, fold_blocks=1, **common)
            self.ss_osd = OsdSolver(Hss, osd_method, osd_order, osd_threads)
        if mode == "bpd_detector":
            # reference BPDetectorCorrect (_experiment.py:128-151): BP (no OSD) on the
            # DEM's fault check matrix with its fault priors.  The sampler's
            # spacetime syndrome is the DEM's detector vector; the readout-flip
            # faults (the DEM's last n columns) carry fault-map columns Lz[:, j], so
            # the readout placed there reproduces the observables and the fused
            # check any(F (v ^ x)) = any(obs ^ F x) is the reference's failure flag.
            if noise is None or getattr(noise, "kind", "") != "depolarizing":
                raise NotImplementedError("bpd_detector builds its DEM for depolarizing_noise(p, pm) only")
            from .dem import DetectorSpacetimeCode, storage_experiment_dem
            if R >= 2:
                import warnings
                warnings.warn("bpd_detector at rounds >= 2 decodes the storage experiment's Z-sector DEM, not Stim's "
                              "two-sector circuit DEM the reference uses (_experiment.py:174,186): its LER is not "
                              "reference-equivalent (unpinned without Stim; dem.storage_experiment_dem)",
                              RuntimeWarning, stacklevel=2)
            self.dem = DetectorSpacetimeCode(storage_experiment_dem(self.H, self.L, R, noise.p, noise.pm))
            fmap = self.dem.fault_map.toarray() % 2
            self.n_faults = self.dem.fault_priors.size
            self.det = Decoder(self.dem.fault_check_matrix, self.dem.fault_priors,
                               logicals=fmap if fmap.shape[0] else None, **common)
        # a plain-H decoder for the sampler
        self.sampler_graph = Decoder(self.H, 0.01, device=self.device)

    # ----------------------------------------------------------- helpers
    def decoders(self):
        """The BP decoders this pipeline launches (for the timing ring)."""
        return [d for d in (getattr(self, k, None) for k in ("st", "fin", "ss", "det")) if d is not None]

    def launches_per_batch(self, dec) -> int:
        """Decode calls `dec` receives per run(): the single-shot decoder runs
        once per syndrome round, every other decoder once."""
        return self.R if dec is getattr(self, "ss", None) else 1

    def _fail_host(self, readout, corr):
        if self.L.shape[0] == 0:
            return np.zeros(readout.shape[0], bool)
        return ((np.asarray(((readout ^ corr).astype(np.int64)) @ self.L.T.astype(np.int64))) % 2).any(axis=1)

    def _osd_fix(self, dec, osd, syn_d, status_d, llr_d, B):
        """OSD for shots whose BP did not converge; returns (idx, osdw) on host."""
        torch = _torch()
        bad = torch.nonzero((status_d & 1) == 0).flatten()
        if bad.numel() == 0:
            return None, None
        idx = bad.cpu().numpy()
        s = syn_d.index_select(0, bad).cpu().numpy()
        llr = llr_d.index_select(0, bad).double().cpu().numpy()
        _, ow = osd.solve(s, llr)
        return idx, ow

    def run(self, syn, readout, want_corrections: bool = False) -> BatchResult:
        torch = _torch()
        B = syn.shape[0]
        dev = syn.device
        u8 = dict(dtype=torch.uint8, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        n, m, R = self.n, self.m, self.R
        iters = torch.zeros(B, **i32)
        status = torch.zeros(B, **u8)
        fail = torch.zeros(B, **u8)
        steps = torch.zeros(B, **i32)
        corr = torch.zeros((B, n), **u8)
        host_fix = None  # (idx, corrections) applied on host
        mode = self.mode
        if mode in ("bp", "bposd"):
            need_llr = mode == "bposd"
            llr = torch.empty((B, self.st.n), dtype=torch.float32 if self.st.precision == _abi.QD_F32
                              else torch.float64, device=dev) if need_llr else None
            self.st.decode_device(B, syn=syn, readout=readout, corr=corr, llr=llr, iters=iters, status=status,
                                  fail=fail)
            if need_llr and self.st.osd_device_supported:
                self.st.osd_device(B, llr=llr, method=self.osd_method, order=self.osd_order, syn=syn, status=status,
                                   readout=readout, corr=corr, fail=fail)
            elif need_llr:
                idx, ow = self._osd_fix(self.st, self.st_osd, syn, status, llr, B)
                if idx is not None:
                    fold = np.zeros((idx.size, n), np.uint8)
                    for t in range(R + 1):
                        fold ^= ow[:, t * n:(t + 1) * n]
                    host_fix = (idx, fold)
        elif mode in ("bposd_hybrid", "bpssf_hybrid"):
            c1 = torch.empty((B, n), **u8)
            self.st.decode_device(B, syn=syn, corr=c1, iters=iters)
            if mode == "bpssf_hybrid":
                self.fin.decode_device(B, base=c1, readout=readout, corr=corr, status=status, ssf_steps=steps,
                                       fail=fail, syn_flags=3)
            else:
                llr = torch.empty((B, n), dtype=torch.float32 if self.fin.precision == _abi.QD_F32
                                  else torch.float64, device=dev)
                self.fin.decode_device(B, base=c1, readout=readout, corr=corr, llr=llr, status=status, fail=fail,
                                       syn_flags=3)
                bad = torch.nonzero((status & 1) == 0).flatten() if not self.fin.osd_device_supported else None
                if bad is None:
                    self.fin.osd_device(B, llr=llr, method=self.osd_method, order=self.osd_order, syn_flags=3,
                                        status=status, base=c1, readout=readout, corr=corr, fail=fail)
                elif bad.numel():
                    idx = bad.cpu().numpy()
                    v = (readout.index_select(0, bad) ^ c1.index_select(0, bad)).cpu().numpy()
                    s2 = ((self.H @ v.T).T % 2).astype(np.uint8)
                    _, ow = self.fin_osd.solve(s2, llr.index_select(0, bad).double().cpu().numpy())
                    host_fix = (idx, c1.index_select(0, bad).cpu().numpy() ^ ow)
        elif mode == "bpssf":
            self.fin.decode_device(B, syn=syn, readout=readout, corr=corr, iters=iters, status=status,
                                   ssf_steps=steps, fail=fail)
        elif mode == "bpd_detector":
            v = torch.zeros((B, self.n_faults), **u8)
            v[:, self.n_faults - n:] = readout
            self.det.decode_device(B, syn=syn, readout=v, iters=iters, status=status, fail=fail)
        elif mode == "bposd_single_shot":
            acc = torch.zeros((B, n), **u8)
            raw = torch.zeros((B, m), **u8)
            sv = syn.view(B, R + 1, m)
            Hss_n = self.ss.n
            for t in range(R):
                raw ^= sv[:, t]
                st_t = torch.zeros(B, **u8)
                llr = torch.empty((B, Hss_n), dtype=torch.float32 if self.ss.precision == _abi.QD_F32
                                  else torch.float64, device=dev)
                new_acc = torch.empty((B, n), **u8)
                s_in = raw.contiguous()
                self.ss.decode_device(B, syn=s_in, base=acc, corr=new_acc, llr=llr, status=st_t, syn_flags=1)
                bad = torch.nonzero((st_t & 1) == 0).flatten() if not self.ss.osd_device_supported else None
                if bad is None:
                    self.ss.osd_device(B, llr=llr, method=self.osd_method, order=self.osd_order, syn=s_in,
                                       syn_flags=1, status=st_t, base=acc, corr=new_acc)
                elif bad.numel():
                    a_h = acc.index_select(0, bad).cpu().numpy()
                    s_h = s_in.index_select(0, bad).cpu().numpy() ^ ((self.H @ a_h.T).T % 2).astype(np.uint8)
                    _, ow = self.ss_osd.solve(s_h, llr.index_select(0, bad).double().cpu().numpy())
                    new_acc[bad] = torch.from_numpy(a_h ^ ow[:, :n]).to(dev)
                acc = new_acc
            llr = torch.empty((B, n), dtype=torch.float32 if self.fin.precision == _abi.QD_F32 else torch.float64,
                              device=dev)
            self.fin.decode_device(B, base=acc, readout=readout, corr=corr, llr=llr, iters=iters, status=status,
                                   fail=fail, syn_flags=3)
            bad = torch.nonzero((status & 1) == 0).flatten() if not self.fin.osd_device_supported else None
            if bad is None:
                self.fin.osd_device(B, llr=llr, method=self.osd_method, order=self.osd_order, syn_flags=3,
                                    status=status, base=acc, readout=readout, corr=corr, fail=fail)
            elif bad.numel():
                idx = bad.cpu().numpy()
                a_h = acc.index_select(0, bad).cpu().numpy()
                v = readout.index_select(0, bad).cpu().numpy() ^ a_h
                s2 = ((self.H @ v.T).T % 2).astype(np.uint8)
                _, ow = self.fin_osd.solve(s2, llr.index_select(0, bad).double().cpu().numpy())
                host_fix = (idx, a_h ^ ow)
        fail_h = fail.cpu().numpy().astype(bool)
        corr_h = corr.cpu().numpy() if (want_corrections or host_fix is not None) else None
        if host_fix is not None:
            idx, c = host_fix
            corr_h[idx] = c
            fail_h[idx] = self._fail_host(readout.index_select(0, torch.from_numpy(idx).to(dev)).cpu().numpy(), c)
        return BatchResult(fail=fail_h, bp_converged=int((status & 1).sum().item()),
                           iters_sum=int(iters.to(torch.int64).sum().item()),
                           ssf_steps_sum=int(steps.to(torch.int64).sum().item()),
                           corrections=corr_h if want_corrections else None)


# ------------------------------------------------------------------ per-shot API
class _PerShot:
    """Reference-style wrapper: ``readout_correction(history, readout)`` for one
    shot (history(t) = Z-check outcomes of round t), via a batch of 1."""

    mode = "bposd"

    def __init__(self, code, rounds: int, bp_osd_options: Dict, priors: Tuple[float, float], **kw):
        self._code = code
        self._rounds = int(rounds)
        self._pipe = BatchPipeline(code, rounds, self.mode, bp_osd_options, priors, **kw)

    def readout_correction(self, history: Callable[[int], np.ndarray], readout) -> np.ndarray:
        torch = _torch()
        H = self._pipe.H
        R = self._rounds
        readout = np.asarray(readout, dtype=np.uint8) % 2
        rows = [np.asarray(history(t), dtype=np.uint8) % 2 for t in range(R)]
        from .spacetime import spacetime_syndrome_batch
        hist = np.stack(rows)[None] if R else np.zeros((1, 0, H.shape[0]), np.uint8)
        syn = spacetime_syndrome_batch(R, H, hist, readout[None])
        dev = torch.device("cuda", self._pipe.device)
        res = self._pipe.run(torch.from_numpy(syn).to(dev), torch.from_numpy(readout[None].copy()).to(dev),
                             want_corrections=True)
        return res.corrections[0].astype(np.int64)


class BPOSDCorrect(_PerShot):
    mode = "bposd"


class BPOSDHybridCorrect(_PerShot):
    mode = "bposd_hybrid"


class BPOSDCorrectSingleShot(_PerShot):
    mode = "bposd_single_shot"


class BPSSFCorrect(_PerShot):
    mode = "bpssf"


class BPSSFHybridCorrect(_PerShot):
    mode = "bpssf_hybrid"


class BPDetectorCorrect:
    """Reference ``BPDetectorCorrect`` (_experiment.py:128-151): BP on the fault
    check matrix of a detector error model (DEM text or dem.DetectorErrorModel);
    ``readout_correction(detector_string)`` returns the corrected observables."""

    def __init__(self, detector_error_model, bp_osd_options: Dict, *, device: int = 0, precision: str = "f64"):
        from .dem import DetectorSpacetimeCode
        self._detector_spacetime_code = DetectorSpacetimeCode(detector_error_model)
        o = bp_osd_options
        c = self._detector_spacetime_code
        self._bpd = Decoder(c.fault_check_matrix, c.fault_priors, method=o.get("bp_method", "ps"), precision=precision,
                            max_iter=int(o.get("max_iter", 0) or 0), ms_scaling=float(o.get("ms_scaling_factor", 0.0)),
                            device=device)

    def readout_correction(self, detector_string) -> np.ndarray:
        c = self._detector_spacetime_code
        d = c.fault_check_matrix.shape[0]
        s = np.asarray(detector_string, dtype=np.uint8) % 2
        fault_set = self._bpd.decode(s[:d][None], want=("x",))["x"][0]
        return ((s[d:].astype(np.int64) + c.fault_map.astype(np.int64) @ fault_set) % 2).astype(np.int64)


# ------------------------------------------------------------------ simulation
def _steps(checks):
    def mx(a):
        a = sp.csr_matrix(a)
        return max(int(a.sum(axis=0).max()), int(a.sum(axis=1).max()))
    return mx(checks.x), mx(checks.z)


def run_simulation(samples, code, meas_prior, data_prior, noise_model, noise_model_args, bp_osd_options, rounds,
                   decoder_mode, *, seed: int = DEFAULT_SEED, stream_id: int = 0, shot0: int = 0, device: int = 0,
                   batch: int = 1 << 18, precision: str = "f64", stats: dict | None = None):
    """Sample and decode `samples` shots on one GPU; returns a bool ndarray of
    logical-failure flags (reference run_simulation, _experiment.py:154-210,
    which returns a list of the same flags)."""
    torch = _torch()
    x_steps, z_steps = _steps(code.checks)
    sim = build_storage_simulation(rounds, noise_model(**noise_model_args), code, use_x_logicals=False)
    mp = meas_prior(x_steps, z_steps)
    dp = data_prior(x_steps, z_steps)
    pipe = BatchPipeline(code, rounds, decoder_mode, bp_osd_options, (dp, mp), device=device, precision=precision,
                         noise=noise_model(**noise_model_args))
    out = np.zeros(samples, dtype=bool)
    agg = {"bp_converged": 0, "iters_sum": 0, "ssf_steps_sum": 0}
    with torch.cuda.device(device):
        for start in range(0, samples, batch):
            b = min(batch, samples - start)
            syn, rd = sim.sample_device(pipe.sampler_graph, b, seed, stream_id, shot0 + start)
            res = pipe.run(syn, rd)
            out[start:start + b] = res.fail
            agg["bp_converged"] += res.bp_converged
            agg["iters_sum"] += res.iters_sum
            agg["ssf_steps_sum"] += res.ssf_steps_sum
    if stats is not None:
        stats.update(agg)
    return out


def add_bposd_args(parser):
    """BP+OSD options (reference add_bposd_args, _experiment.py:213-219)."""
    parser.add_argument("--bposd_max_iter", type=lambda x: int(x) if x is not None else None,
                        help="Maximum number of iterations for BP. Default is the number of qubits in the code",
                        default=None)
    parser.add_argument("--bposd_bp_method", choices=["ps", "ms", "msl"],
                        help="BP method (product-sum, min-sum, min-sum log)", default="ps")
    parser.add_argument("--bposd_ms_scaling_factor", type=float,
                        help="Min sum scaling factor. Use variable scaling factor method if 0", default=0)
    parser.add_argument("--bposd_osd_method", choices=["osd_e", "osd_cs", "osd0"], help="OSD method", default="osd_cs")
    parser.add_argument("--bposd_osd_order", type=int, help="OSD search depth", default=7)


def unpack_bposd_args(parsed_args, code):
    """Reference unpack_bposd_args (_experiment.py:221-229): max_iter defaults to
    the number of qubits."""
    return {
        "max_iter": parsed_args.bposd_max_iter if parsed_args.bposd_max_iter is not None else code.checks.num_qubits,
        "bp_method": parsed_args.bposd_bp_method,
        "ms_scaling_factor": parsed_args.bposd_ms_scaling_factor,
        "osd_method": parsed_args.bposd_osd_method,
        "osd_order": parsed_args.bposd_osd_order,
    }


def load_code(args):
    with Path(args.code).open() as f:
        return read_quantum_code(f, validate_stabilizer_code=True)


# ------------------------------------------------------------------ sweep
def _device_count() -> int:
    try:
        return max(1, _abi.load().qd_device_count())
    except Exception:
        return 1


def _load_checkpoint(path):
    """Rows of a previous run's checkpoint CSV, keyed by (p, config fingerprint)
    (empty when absent)."""
    import pandas as pd
    if not path or not os.path.exists(path) or os.path.getsize(path) == 0:
        return {}
    try:
        df = pd.read_csv(path, float_precision="round_trip", dtype={"config_fp": str})
    except Exception:  # unparseable file: nothing is reused (the next append sets it aside)
        return {}
    if "config_fp" not in df.columns:  # rows without a fingerprint are never reused
        return {}
    return {(float(r["p_ph"]), str(r["config_fp"])): r.to_dict() for _, r in df.iterrows()
            if isinstance(r["config_fp"], str)}


def _config_fingerprint(code, rounds, mode, bp_osd_options, precision, seed, samples, point_index,
                        noise=None) -> str:
    """Everything a point's failure count depends on besides p: the check
    matrices and logicals, the decoder configuration, the sampler stream
    (seed, point index = Philox stream id, sample count) and the point's noise
    configuration ``noise = (noise model, noise_model_args(p), data prior,
    measurement prior)``: the sampler's event probabilities and the BP priors
    are built from exactly those."""
    import hashlib
    h = hashlib.sha1()
    for M in (code.checks.x, code.checks.z, code.logicals.x, code.logicals.z):
        A = sp.csr_matrix(M)
        A.sort_indices()
        h.update(repr(A.shape).encode())
        h.update(np.ascontiguousarray(A.indptr, dtype=np.int64).tobytes())
        h.update(np.ascontiguousarray(A.indices, dtype=np.int64).tobytes())
    h.update(repr((int(rounds), str(mode), sorted((k, str(v)) for k, v in bp_osd_options.items()), str(precision),
                   int(seed), int(samples), int(point_index))).encode())
    if noise is not None:
        model, model_args, dp, mp = noise
        name = f"{getattr(model, '__module__', '')}.{getattr(model, '__qualname__', repr(model))}"
        h.update(repr((name, sorted((str(k), repr(v)) for k, v in dict(model_args).items()))).encode())
        for prior in (dp, mp):
            h.update(np.ascontiguousarray(np.atleast_1d(np.asarray(prior, dtype=np.float64))).tobytes())
            h.update(b"|")
    return h.hexdigest()[:16]


def _append_checkpoint_row(path, point) -> None:
    """Append one finished point to the checkpoint CSV.  A file written with a
    different column set (an older format, other decoder options) is rewritten
    with the union of the columns first, so every row stays parseable and the
    sweep stays resumable (missing cells are empty)."""
    import pandas as pd
    row = pd.DataFrame.from_records([point])
    if not os.path.exists(path) or os.path.getsize(path) == 0:
        row.to_csv(path, mode="w", header=True, index=False, float_format="%.17g")
        return
    with open(path) as f:
        header = f.readline().rstrip("\n").split(",")
    if header == list(row.columns):
        row.to_csv(path, mode="a", header=False, index=False, float_format="%.17g")
        return
    try:
        old = pd.read_csv(path, float_precision="round_trip", dtype={"config_fp": str})
    except Exception:  # unreadable (e.g. rows wider than their header): keep it aside, start afresh
        os.replace(path, path + ".unreadable")
        row.to_csv(path, mode="w", header=True, index=False, float_format="%.17g")
        return
    cols = list(old.columns) + [c for c in row.columns if c not in old.columns]
    merged = pd.concat([old.reindex(columns=cols), row.reindex(columns=cols)], ignore_index=True)
    tmp = path + ".tmp"
    merged.to_csv(tmp, mode="w", header=True, index=False, float_format="%.17g")
    os.replace(tmp, path)


class ShardError(RuntimeError):
    """A shot range that failed twice (once, then once more in a fresh worker)."""

    def __init__(self, p_ph, device, lo, hi, cause):
        super().__init__(f"p_sweep shard failed twice: p={p_ph!r}, device {device}, shots [{lo}, {hi}): {cause!r}")
        self.p_ph, self.device, self.lo, self.hi, self.cause = p_ph, device, lo, hi, cause


def device_error(e: BaseException) -> bool:
    """True for failures of the device itself (a HIP error from the library --
    codes <= -100, a failed launch or allocation -- or from torch): a retry on
    the same device would only meet the same sticky error."""
    from ._abi import QdecError
    if isinstance(e, QdecError):
        return getattr(e, "rc", 0) <= -100
    msg = str(e)
    return isinstance(e, RuntimeError) and ("HIP error" in msg or "hipError" in msg)


def run_shards(shards, work, p_ph=None, retries: int = 1):
    """Run work(device, lo, hi, attempt) -> counters for every (device, lo, hi)
    shard, one host thread per shard (each blocks on its own device's copies),
    and sum the counters.  A shard that raises a host-side exception is run
    again in a fresh worker thread on the same device (its handles rebuilt by
    `work` when attempt > 0; never a re-exec of a process that touched the GPU),
    up to `retries` times; then ShardError names the point and the failed shot
    range.  A device error (device_error) is not retried: ShardError at once.
    The reference fan-out (misc/p_sweep.py:24-40, Pool.starmap) aborts the sweep
    on any worker exception."""
    from concurrent.futures import ThreadPoolExecutor

    def attempt(i, k):
        d, lo, hi = shards[i]
        return work(d, lo, hi, k)

    results = [None] * len(shards)
    pending = list(range(len(shards)))
    for k in range(retries + 1):
        errors = {}
        if len(pending) == 1 and k == 0:  # the common 1-device case: no thread
            try:
                results[pending[0]] = attempt(pending[0], 0)
            except Exception as e:  # noqa: BLE001 - retried below, then reported with its range
                errors[pending[0]] = e
        else:
            with ThreadPoolExecutor(max_workers=len(pending)) as ex:  # fresh threads every attempt
                futs = {i: ex.submit(attempt, i, k) for i in pending}
                for i, f in futs.items():
                    try:
                        results[i] = f.result()
                    except Exception as e:  # noqa: BLE001
                        errors[i] = e
        if not errors:
            break
        pending = sorted(errors)
        if k == retries or any(device_error(e) for e in errors.values()):
            i = pending[0]
            i = next((j for j in pending if device_error(errors[j])), i)
            d, lo, hi = shards[i]
            raise ShardError(p_ph, d, lo, hi, errors[i]) from errors[i]
    n = max(len(r) for r in results)
    return [sum(r[j] for r in results) for j in range(n)]


HBM_PEAK_BYTES_S = 8.0e12  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def p_sweep(samples, p_values, noise_model, noise_model_args, meas_prior, data_prior, *, gpus: int | None = None,
            devices=None, seed: int = DEFAULT_SEED, batch: int = 1 << 18, precision: str = "f64",
            checkpoint: str | None = None, **kwargs):
    """Sweep the physical error rate (reference p_sweep, misc/p_sweep.py:17-40).
    Shots are sharded over `gpus` devices by index (shard d decodes a
    contiguous shot range); exactly `samples` shots per point.  `devices`
    (a list of device ordinals, repeats allowed) overrides `gpus`: one shard per
    entry.  BP runs in `precision` (default f64, ldpc v1's message precision);
    every row records it.  A failed shard is retried once in a fresh worker
    thread (run_shards); a second failure raises ShardError with its range.

    Per point, besides the reference's columns: shots_per_s, bp_converged_frac,
    iters_mean, ssf_steps_mean, and from the library's HIP-event timing ring
    kernel_ms (summed over shards and decode stages), hbm_bytes (the compulsory
    per-shot I/O: syndrome + readout in, failure flag out) and
    hbm_roofline_frac = hbm_bytes / kernel time / HBM peak (summed kernel time:
    shards on distinct devices overlap, so this is per device-second).

    checkpoint: CSV path; each finished point is appended to it at once, and a
    restarted sweep reuses a row only when its p and its configuration
    fingerprint match (code, logicals, rounds, mode, BP/OSD options, precision,
    seed, sample count and the point index, which is the point's Philox stream
    id), since a recomputed point would then be identical.  The reference
    writes its CSV only at the end (misc/p_sweep.py:78)."""
    import pandas as pd
    torch = _torch()
    done = _load_checkpoint(checkpoint)
    devs = [int(d) for d in devices] if devices else list(range(gpus or _device_count()))
    ndev = len(devs)
    code = kwargs["code"]
    rounds = kwargs["rounds"]
    mode = kwargs["decoder_mode"]
    bp_osd_options = kwargs["bp_osd_options"]
    x_steps, z_steps = _steps(code.checks)
    data = []
    for pi, p_ph in enumerate(p_values):
        nm_args = noise_model_args(p_ph)
        dp = data_prior(p_ph, x_steps, z_steps)
        mp = meas_prior(p_ph, x_steps, z_steps)
        fp = _config_fingerprint(code, rounds, mode, bp_osd_options, precision, seed, samples, pi,
                                 noise=(noise_model, nm_args, dp, mp))
        prev = done.get((float(p_ph), fp))
        if prev is not None:
            data.append(prev)
            continue
        t0 = time.perf_counter()
        nm = noise_model(**nm_args)
        sim = build_storage_simulation(rounds, nm, code, use_x_logicals=False)

        def pipeline(d):
            return BatchPipeline(code, rounds, mode, bp_osd_options, (dp, mp), device=d, precision=precision,
                                 noise=nm)
        pipes = [pipeline(d) for d in devs]
        per = math.ceil(samples / ndev)
        shards = [(i, i * per, min(samples, (i + 1) * per)) for i in range(ndev)]

        def shard(i, lo, hi, attempt):
            """Shard i's contiguous shot range on device devs[i]; returns its
            counters (failures, converged, iterations, SSF steps, kernel ms)."""
            d = devs[i]
            if attempt > 0:  # a retry frees the failed pipeline's handles, then rebuilds them
                for dec in pipes[i].decoders() + [pipes[i].sampler_graph]:
                    dec.close()
                pipes[i] = pipeline(d)
            pipe = pipes[i]
            nb = max(1, -(-(hi - lo) // batch))
            decs = pipe.decoders()
            for dec in decs:  # one ring slot per decode call (ss: one per round)
                dec.set_timing(nb * pipe.launches_per_batch(dec))
            acc = [0, 0, 0, 0, 0.0]
            with torch.cuda.device(d):
                for start in range(lo, hi, batch):
                    b = min(batch, hi - start)
                    syn, rd = sim.sample_device(pipe.sampler_graph, b, seed, pi, start)
                    res = pipe.run(syn, rd)
                    acc[0] += int(res.fail.sum())
                    acc[1] += res.bp_converged
                    acc[2] += res.iters_sum
                    acc[3] += res.ssf_steps_sum
                torch.cuda.synchronize(d)
            for dec in decs:
                bp, ssf = dec.read_timing()
                acc[4] += float(bp.sum() + ssf.sum())
            return acc

        failures, conv, iters, ssf, kernel_ms = run_shards(shards, shard, p_ph=p_ph)
        runtime = time.perf_counter() - t0
        hbm = samples * ((rounds + 1) * pipes[0].m + pipes[0].n + 1)
        point = {"p_ph": p_ph, "failures": failures, "samples": samples, "walltime": runtime, **kwargs,
                 **bp_osd_options, "gpus": ndev, "shots_per_s": samples / runtime if runtime > 0 else float("nan"),
                 "bp_converged_frac": conv / samples if samples else 0.0,
                 "iters_mean": iters / samples if samples else 0.0,
                 "ssf_steps_mean": ssf / samples if samples else 0.0,
                 "kernel_ms": kernel_ms, "hbm_bytes": hbm,
                 "hbm_roofline_frac": hbm / (kernel_ms * 1e-3) / HBM_PEAK_BYTES_S if kernel_ms > 0 else float("nan")}
        del point["code"]
        del point["bp_osd_options"]
        point["seed"] = seed
        point["precision"] = precision
        point["point_index"] = pi
        point["config_fp"] = fp
        if mode == "bpd_detector" and rounds >= 2:
            point["dem_sector"] = "z_only_unpinned"  # see BatchPipeline's warning / dem.storage_experiment_dem
        data.append(point)
        if checkpoint:
            _append_checkpoint_row(checkpoint, point)
    return pd.DataFrame.from_records(data)


_SWEEP_RE = re.compile(r"^\s*[(](.+),(.+),(.+)[)]\s*$")


def parse_sweep_spec(x: str) -> Tuple[float, float, int]:
    """'(a, b, c)' -> (float, float, int), a <= b, c > 0 (misc/p_sweep.py:43-55)."""
    r = _SWEEP_RE.match(x)
    if r is None:
        raise RuntimeError("Unable to parse sweep specification, expecting (a, b, c) where a,b : float, c : int, "
                           "a<=b, and c > 0. Ex: (0.3, 1e3, 10)")
    lo, hi, pts = float(r.group(1)), float(r.group(2)), int(r.group(3))
    if pts <= 0 or lo > hi:
        raise RuntimeError("Number of points non-positive or lower bound exceeded upper bound")
    return lo, hi, pts


def p_sweep_main(noise_model_args, noise_model, meas_prior, data_prior):
    """CLI of the sweep (reference p_sweep_main, misc/p_sweep.py:57-78); extra
    flags: --gpus, --seed, --batch, --precision, --checkpoint; extra decoder
    modes bpssf, bpssf_hybrid, bp."""
    parser = ArgumentParser(description="Perform a parallelized sweep in the physical error rate for the given "
                                        "quantum code under BP+OSD / BP+SSF on MI355X")
    parser.add_argument("code", type=Path)
    parser.add_argument("--samples", type=int, help="Number of samples to take")
    parser.add_argument("--p_sweep", type=parse_sweep_spec,
                        help="Specify lower and upper bounds of the sweep + number of points in the form "
                             "(lower, upper, points)")
    parser.add_argument("--rounds", type=int, help="Number of rounds of syndrome extraction", default=1)
    parser.add_argument("--decoder_mode", choices=DECODER_MODES, default="bposd",
                        help="Operate decoder in BP+OSD, BP+OSD (single shot), hybrid BP + (BP+OSD), or BP+SSF")
    parser.add_argument("--linspace", type=bool, default=False,
                        help="Perform the sweep with linearly spaced points. The default is uniform spacing in log "
                             "space")
    add_bposd_args(parser)
    parser.add_argument("--gpus", type=int, default=None, help="GPUs to shard shots over (default: all visible)")
    parser.add_argument("--devices", type=lambda v: [int(x) for x in v.split(",") if x.strip()], default=None,
                        help="comma-separated device ordinals, one shot shard each (repeats allowed; overrides --gpus)")
    parser.add_argument("--seed", type=int, default=DEFAULT_SEED, help="sampler seed (counter-based Philox)")
    parser.add_argument("--batch", type=int, default=1 << 18, help="shots per device launch")
    parser.add_argument("--precision", choices=["f32", "f64"], default="f64",
                        help="BP message precision (default f64, as ldpc v1; f32 is the faster stated-tolerance variant)")
    parser.add_argument("--checkpoint", type=str, default=None,
                        help="CSV that each finished point is appended to; finished points are skipped on restart")
    args = parser.parse_args(sys.argv[1:])
    code = load_code(args)
    bp_osd_options = unpack_bposd_args(args, code)
    sweep = np.linspace(*args.p_sweep) if args.linspace else np.geomspace(*args.p_sweep)
    result = p_sweep(samples=args.samples, code=code, rounds=args.rounds, noise_model=noise_model,
                     noise_model_args=noise_model_args, meas_prior=meas_prior, data_prior=data_prior,
                     p_values=sweep, decoder_mode=args.decoder_mode, bp_osd_options=bp_osd_options,
                     gpus=args.gpus, devices=args.devices, seed=args.seed, batch=args.batch, precision=args.precision,
                     checkpoint=args.checkpoint)
    result.to_csv(sys.stdout)
    return result
