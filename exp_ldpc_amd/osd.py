"""Ordered-statistics decoding stage, host side (C++ in libqdec_hip.so,
qd_osd_batch).  The batched pipelines use the GPU version
(Decoder.osd_device -> qd_osd_batch_device, csrc/qdec_osd.hip, bit-identical)
whenever the graph fits it (m <= 384, n < 1024); this host stage serves the
single-shot ldpc-compatible API and larger graphs.

Post-processes the BP soft output of shots BP did not converge on, as ldpc v1's
``bposd_decoder`` does (reference call sites python/qldpc/misc/_experiment.py:23,
37, 77, 96).  Methods: 'osd0', 'osd_e' (exhaustive over the first ``order``
non-pivot columns), 'osd_cs' (combination sweep: all single non-pivot columns +
pairs among the first ``order``).  See csrc/qdec_osd.cpp for the exact spec.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi
from .decoder import as_csr01

OSD_METHODS = {"osd0": 0, "osd_e": 1, "osd_cs": 2}
_METHODS = OSD_METHODS


class OsdSolver:
    def __init__(self, H, method: str = "osd_cs", order: int = 0, nthreads: int = 0):
        self._lib = _abi.load()
        H = as_csr01(H)
        self.m, self.n = H.shape
        self._rp = np.ascontiguousarray(H.indptr, dtype=np.int32)
        self._ci = np.ascontiguousarray(H.indices, dtype=np.int32)
        if method not in _METHODS:
            raise ValueError(f"unknown OSD method {method!r}")
        self.method = _METHODS[method]
        self.order = int(order)
        self.nthreads = int(nthreads or os.environ.get("QDEC_OSD_THREADS", "0") or 0)

    def solve(self, syndromes, llrs):
        """syndromes uint8[B, m], llrs float[B, n] -> (osd0 uint8[B, n], osdw uint8[B, n])."""
        syn = np.ascontiguousarray(syndromes, dtype=np.uint8).reshape(-1, self.m)
        llr = np.ascontiguousarray(llrs, dtype=np.float64).reshape(-1, self.n)
        B = syn.shape[0]
        o0 = np.zeros((B, self.n), np.uint8)
        ow = np.zeros((B, self.n), np.uint8)
        rc = self._lib.qd_osd_batch(self.m, self.n, _abi.ptr(self._rp), _abi.ptr(self._ci), self.method, self.order,
                                    B, _abi.ptr(syn), _abi.ptr(llr), _abi.ptr(o0), _abi.ptr(ow), self.nthreads)
        if rc != 0:
            raise _abi.QdecError(f"qd_osd_batch failed ({rc}): {self._lib.qd_osd_last_error().decode()}")
        return o0, ow
