"""ctypes wrapper for oracle/libqdec_oracle.so (test infrastructure only)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QDEC_ORACLE_LIB") or os.path.join(HERE, "libqdec_oracle.so")  # env: sanitizer variant

_p = C.c_void_p
_i32 = C.c_int32
_i64 = C.c_int64


def build(force: bool = False) -> str:
    """(Re)build with make; a no-op when the library is up to date."""
    cmd = ["make", "-C", HERE, "-s"] + (["-B"] if force else [])
    subprocess.run(cmd, check=True)
    return LIB_PATH


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_p)


class OracleLib:
    def __init__(self, path: str = LIB_PATH):
        self.lib = C.CDLL(path)
        f = self.lib.qdo_decode_batch
        f.restype = _i32
        f.argtypes = [_i32, _i32, _p, _p, _p, _i32, _i32, _i32, C.c_double, _i32, _i32,
                      _i32, _p, _p, _i32, _i32, _i32, _p, _i64, _p, _p, _p, _i32,
                      _p, _p, _p, _p, _p, _p, _p, _i32, _i32]
        s = self.lib.qdo_sample_storage
        s.restype = _i32
        s.argtypes = [_i32, _i32, _p, _p, _i32, C.c_double, C.c_double, C.c_uint32, C.c_uint32,
                      _i64, _i64, _p, _p, _i32]
        ph = self.lib.qdo_philox4x32_10
        ph.restype = None
        ph.argtypes = [_p, _p, _p]
        o = self.lib.qdo_osd_batch
        o.restype = _i32
        o.argtypes = [_i32, _i32, _p, _p, _i64, _p, _p, _i32, _i32, _p, _p, _i32]
        th = self.lib.qdo_threshold
        th.restype = C.c_uint32
        th.argtypes = [C.c_double]

    def decode(self, H, probs, syn=None, *, method="ms", precision="f64", max_iter=0, ms_scaling=0.0,
               ssf=False, ssf_max_steps=0, gens=None, n_data=None, fold_blocks=1, lz=None,
               base=None, readout=None, syn_flags=0, B=None, want_llr=True, nthreads=0, ssf_impl="brute"):
        """Decode a batch; returns a dict of numpy arrays (same contract as
        exp_ldpc_amd.decoder.Decoder.decode_batch)."""
        import scipy.sparse as sp
        H = sp.csr_matrix(H)
        H.sort_indices()
        m, n = H.shape
        rp = np.ascontiguousarray(H.indptr, dtype=np.int32)
        ci = np.ascontiguousarray(H.indices, dtype=np.int32)
        probs = np.ascontiguousarray(np.broadcast_to(np.asarray(probs, dtype=np.float64), (n,)))
        if n_data is None:
            n_data = n
        if B is None:
            B = syn.shape[0] if syn is not None else readout.shape[0]
        syn = None if syn is None else np.ascontiguousarray(syn, dtype=np.uint8).reshape(B, m)
        base = None if base is None else np.ascontiguousarray(base, dtype=np.uint8).reshape(B, n_data)
        readout = None if readout is None else np.ascontiguousarray(readout, dtype=np.uint8).reshape(B, n_data)
        if gens is not None:
            G = sp.csr_matrix(gens)
            G.sort_indices()
            gp = np.ascontiguousarray(G.indptr, dtype=np.int32)
            gi = np.ascontiguousarray(G.indices, dtype=np.int32)
            ng = G.shape[0]
        else:
            gp = gi = None
            ng = 0
        k = 0
        lz_sparse = None
        if lz is not None and sp.issparse(lz):
            # sparse logicals (thousands of them on the config-5 code): the C loop
            # is skipped and the check any(Lz (readout ^ corr)) (_experiment.py:209)
            # is evaluated below on the oracle's own corrections
            lz_sparse = sp.csr_matrix(lz)
            lz = None
        if lz is not None:
            lz = np.ascontiguousarray(np.asarray(lz) % 2, dtype=np.uint8)
            k = lz.shape[0]
        out = {
            "x": np.zeros((B, n), np.uint8), "corr": np.zeros((B, n_data), np.uint8),
            "llr": np.zeros((B, n), np.float64) if want_llr else None,
            "iters": np.zeros(B, np.int32), "status": np.zeros(B, np.uint8),
            "ssf_steps": np.zeros(B, np.int32), "fail": np.zeros(B, np.uint8),
        }
        meth = {"ps": 0, "ms": 1}[method]
        prec = {"f64": 0, "f32": 1}[precision]
        rc = self.lib.qdo_decode_batch(m, n, _ptr(rp), _ptr(ci), _ptr(probs), meth, prec, int(max_iter),
                                       float(ms_scaling), int(bool(ssf)), int(ssf_max_steps), ng, _ptr(gp), _ptr(gi),
                                       int(n_data), int(fold_blocks), k, _ptr(lz), int(B), _ptr(syn), _ptr(base),
                                       _ptr(readout), int(syn_flags), _ptr(out["x"]), _ptr(out["corr"]),
                                       _ptr(out["llr"]), _ptr(out["iters"]), _ptr(out["status"]),
                                       _ptr(out["ssf_steps"]), _ptr(out["fail"]),
                                       {"brute": 0, "fast": 1}[ssf_impl], int(nthreads))
        if rc != 0:
            raise ValueError(f"qdo_decode_batch failed with status {rc}")
        if lz_sparse is not None and readout is not None:
            resid = sp.csr_matrix((readout ^ out["corr"]) & 1)
            out["fail"] = ((lz_sparse @ resid.T).toarray() % 2).any(axis=0).astype(np.uint8)
        return out

    def sample_storage(self, Hz, rounds, p_data, p_meas, seed, stream, shot0, B, nthreads=0):
        import scipy.sparse as sp
        Hz = sp.csr_matrix(Hz)
        Hz.sort_indices()
        m, n = Hz.shape
        rp = np.ascontiguousarray(Hz.indptr, dtype=np.int32)
        ci = np.ascontiguousarray(Hz.indices, dtype=np.int32)
        syn = np.zeros((B, (rounds + 1) * m), np.uint8)
        rd = np.zeros((B, n), np.uint8)
        rc = self.lib.qdo_sample_storage(m, n, _ptr(rp), _ptr(ci), int(rounds), float(p_data), float(p_meas),
                                         int(seed) & 0xFFFFFFFF, int(stream) & 0xFFFFFFFF, int(shot0), int(B),
                                         _ptr(syn), _ptr(rd), int(nthreads))
        if rc != 0:
            raise ValueError(f"qdo_sample_storage failed with status {rc}")
        return syn, rd

    def osd(self, H, syn, llr, method="osd_cs", order=0, nthreads=0):
        """Compiled OSD (osd_impl.inc) of a batch: returns (osd0, osdw) uint8[B][n]."""
        import scipy.sparse as sp
        H = sp.csr_matrix(H)
        H.sort_indices()
        m, n = H.shape
        syn = np.ascontiguousarray(np.asarray(syn, dtype=np.uint8).reshape(-1, m))
        B = syn.shape[0]
        llr = np.ascontiguousarray(np.asarray(llr, dtype=np.float64).reshape(B, n))
        rp = np.ascontiguousarray(H.indptr, dtype=np.int32)
        ci = np.ascontiguousarray(H.indices, dtype=np.int32)
        o0 = np.zeros((B, n), np.uint8)
        ow = np.zeros((B, n), np.uint8)
        rc = self.lib.qdo_osd_batch(m, n, _ptr(rp), _ptr(ci), int(B), _ptr(syn), _ptr(llr),
                                    {"osd0": 0, "osd_e": 1, "osd_cs": 2}[method], int(order), _ptr(o0), _ptr(ow),
                                    int(nthreads))
        if rc != 0:
            raise ValueError(f"qdo_osd_batch failed with status {rc}")
        return o0, ow

    def philox(self, ctr, key):
        c = np.ascontiguousarray(ctr, dtype=np.uint32)
        k = np.ascontiguousarray(key, dtype=np.uint32)
        o = np.zeros(4, np.uint32)
        self.lib.qdo_philox4x32_10(_ptr(c), _ptr(k), _ptr(o))
        return o

    def threshold(self, p):
        return int(self.lib.qdo_threshold(float(p)))


_LIB = None


def load() -> OracleLib:
    global _LIB
    if _LIB is None:
        build()
        _LIB = OracleLib()
    return _LIB
