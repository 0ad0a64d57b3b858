"""ldpc-v1-compatible decoder objects backed by the HIP library.

Drop-in for the two classes the reference imports at
``python/qldpc/misc/_experiment.py:2`` (``from ldpc import bp_decoder,
bposd_decoder``; third-party ``ldpc`` v1, quantumgizmos/ldpc rev 7909a97d,
pinned at ``overlays/python/ldpc/default.nix:14-22``).  Construction keywords
and defaults follow ldpc v1 (read with ``.get``, unknown keys ignored):

    error_rate, channel_probs, max_iter (0 -> n), bp_method, ms_scaling_factor
    (default 1.0; 0 -> alpha_t = 1 - 2^-t), input_vector_type,
    osd_method, osd_order                                     (bposd_decoder)

plus ``channel_prior`` as an alias of ``channel_probs`` (the reference passes it
at ``_experiment.py:77``).  ``.decode(v)`` accepts a syndrome
(length m) or an error vector (length n, syndrome taken first) and returns a new
int ndarray of length n; afterwards ``.converge``, ``.iter``,
``.log_prob_ratios`` and ``.bp_decoding`` (and ``.osd0_decoding`` /
``.osdw_decoding``) are set as in ldpc.  ``decode_batch`` is the throughput
path.  Extra: ``precision`` ('f64' = ldpc's double arithmetic, the default here;
'f32'), ``device``.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

from .decoder import Decoder, as_csr01, parse_bp_method
from . import _abi

__all__ = ["bp_decoder", "bposd_decoder"]


def _resolve_probs(n, kwargs):
    error_rate = kwargs.get("error_rate", None)
    channel = kwargs.get("channel_probs", None)
    if channel is None:
        channel = kwargs.get("channel_prior", None)
    if channel is not None and not (isinstance(channel, (list, tuple)) and len(channel) == 1 and channel[0] is None):
        channel = np.asarray(channel, dtype=np.float64).reshape(-1)
        if channel.size != n:
            raise ValueError(f"The length of the channel probability vector ({channel.size}) must equal the block "
                             f"length n={n}")
        return channel
    if error_rate is None:
        raise ValueError("Please specify the error channel. Either: 1) error_rate: float or 2) channel_probs: "
                         "array_like")
    return np.full(n, float(error_rate))


class bp_decoder:
    """ldpc v1 ``bp_decoder`` (belief propagation only)."""

    def __init__(self, parity_check_matrix, **kwargs):
        if not (sp.issparse(parity_check_matrix) or isinstance(parity_check_matrix, np.ndarray)):
            raise TypeError("The parity check matrix must be a numpy array or a scipy sparse matrix")
        H = as_csr01(parity_check_matrix)
        self.m, self.n = H.shape
        self.H = H
        max_iter = int(kwargs.get("max_iter", 0) or 0)
        self.max_iter = max_iter if max_iter > 0 else self.n
        self._method = parse_bp_method(kwargs.get("bp_method", 0))
        self.bp_method = "product_sum" if self._method == _abi.QD_PRODUCT_SUM else "minimum_sum_log"
        self.ms_scaling_factor = float(kwargs.get("ms_scaling_factor", 1.0))
        self.input_vector_type = kwargs.get("input_vector_type", -1)
        self.channel_probs = _resolve_probs(self.n, kwargs)
        self.error_rate = kwargs.get("error_rate", None)
        self._dec = Decoder(H, self.channel_probs, method=self._method, precision=kwargs.get("precision", "f64"),
                            max_iter=self.max_iter, ms_scaling=self.ms_scaling_factor,
                            device=int(kwargs.get("device", 0)))
        self.converge = 0
        self.iter = 0
        self.bp_decoding = np.zeros(self.n, dtype=np.uint8)
        self.log_prob_ratios = np.zeros(self.n)

    def update_channel_probs(self, channel) -> None:
        self.channel_probs = np.asarray(channel, dtype=np.float64).reshape(self.n)
        self._dec.set_priors(self.channel_probs)

    def _as_syndromes(self, v):
        v = np.asarray(v)
        squeeze = v.ndim == 1
        v = np.atleast_2d(v)
        if v.shape[1] == self.m and self.input_vector_type != 1:
            syn = v % 2
        elif v.shape[1] == self.n and self.input_vector_type != 0:
            syn = (self.H @ (v.T % 2)).T % 2
        else:
            raise ValueError(f"The input vector is of length {v.shape[1]}; expected a syndrome of length {self.m} "
                             f"or an error vector of length {self.n}")
        return np.ascontiguousarray(syn, dtype=np.uint8), squeeze

    def decode_batch(self, vectors) -> dict:
        """Decode B shots at once; returns {'x', 'llr', 'iters', 'status'}."""
        syn, _ = self._as_syndromes(vectors)
        return self._dec.decode(syn, want=("x", "llr", "iters", "status"))

    def decode(self, input_vector) -> np.ndarray:
        out = self.decode_batch(input_vector)
        self.bp_decoding = out["x"][0].copy()
        self.log_prob_ratios = out["llr"][0].astype(np.float64)
        self.iter = int(out["iters"][0])
        self.converge = int(out["status"][0] & _abi.QD_ST_BP_CONVERGED)
        return self.bp_decoding.astype(np.int64)


class bposd_decoder(bp_decoder):
    """ldpc v1 ``bposd_decoder``: BP, then ordered-statistics decoding when BP
    does not converge (OSD-0 / OSD-E / OSD-CS of order ``osd_order``)."""

    def __init__(self, parity_check_matrix, **kwargs):
        super().__init__(parity_check_matrix, **kwargs)
        method = str(kwargs.get("osd_method", "osd0")).lower()
        aliases = {"osd0": "osd0", "osd_0": "osd0", "0": "osd0", "osd_e": "osd_e", "osde": "osd_e",
                   "exhaustive": "osd_e", "osd_cs": "osd_cs", "osdcs": "osd_cs", "cs": "osd_cs",
                   "combination_sweep": "osd_cs", "1": "osd_e", "2": "osd_cs"}
        if method not in aliases:
            raise ValueError(f"unknown osd_method {method!r}")
        self.osd_method = aliases[method]
        self.osd_order = int(kwargs.get("osd_order", 0))
        if self.osd_method == "osd0":
            self.osd_order = 0
        self.osd0_decoding = np.zeros(self.n, dtype=np.uint8)
        self.osdw_decoding = np.zeros(self.n, dtype=np.uint8)
        from .osd import OsdSolver
        self._osd = OsdSolver(self.H, self.osd_method, self.osd_order)

    def decode_batch(self, vectors) -> dict:
        syn, _ = self._as_syndromes(vectors)
        out = self._dec.decode(syn, want=("x", "llr", "iters", "status"))
        conv = (out["status"] & _abi.QD_ST_BP_CONVERGED).astype(bool)
        out["osd0"] = out["x"].copy()
        out["osdw"] = out["x"].copy()
        bad = np.nonzero(~conv)[0]
        if bad.size:
            o0, ow = self._osd.solve(syn[bad], out["llr"][bad].astype(np.float64))
            out["osd0"][bad] = o0
            out["osdw"][bad] = ow
        return out

    def decode(self, input_vector) -> np.ndarray:
        out = self.decode_batch(input_vector)
        self.bp_decoding = out["x"][0].copy()
        self.log_prob_ratios = out["llr"][0].astype(np.float64)
        self.iter = int(out["iters"][0])
        self.converge = int(out["status"][0] & _abi.QD_ST_BP_CONVERGED)
        self.osd0_decoding = out["osd0"][0].copy()
        self.osdw_decoding = out["osdw"][0].copy()
        return self.osdw_decoding.astype(np.int64)
