"""Batched GPU decoder over one parity-check graph (host side of the C ABI).

``Decoder`` owns a ``qd_graph`` on one device: the matrix, its priors, optional
flip sets (SSF) and logicals (fused failure check).  ``decode`` works on host
numpy arrays (the ldpc-like path, H2D/D2H inside the library); ``decode_device``
works on device-resident torch tensors and only enqueues work on the current
torch stream (the throughput path).

Decode contract (one call = B shots; identical to oracle/qdec_oracle.c):
  1. s = syn (or 0); with syn_flags: s ^= H[:, :n_data] (base ^ readout)
  2. BP (ldpc v1 loops; min-sum log domain or product-sum) until H x = s or max_iter
  3. if ssf and not converged: small-set-flip on the residual s ^ H x
  4. corr = base ^ fold(x),   fold(x)[q] = xor_t x[t*n_data + q]
  5. fail = any_r (Lz[r] . (readout ^ corr)) mod 2
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import scipy.sparse as sp

from . import _abi

__all__ = ["Decoder", "parse_bp_method", "as_csr01", "OPTIONS", "DEFAULT_OPTIONS"]

# per-handle kernel choices (qd_graph_set_option, QD_OPT_* in include/qdec.h);
# every choice gives identical results, they exist for A/B measurements and so
# tests keep each kernel path covered
OPTIONS = {"compact": 1, "triage_it1": 2, "ssf": 3, "lds_kernel": 4, "group_kernel": 5, "ssf_inc": 6,
           "block_wg": 7, "group_mb": 8, "ssf_fuse": 9}
SSF_KERNELS = {"auto": 0, "scan": 1, "scan_gather": 2, "scan_nosplit": 3}  # values of the "ssf" option
# options applied to every Decoder built afterwards (tests patch this dict to
# route pipelines that build their decoders internally through one kernel path)
DEFAULT_OPTIONS: dict = {}

_PS_NAMES = {"ps", "product_sum", "prod_sum", "0", "prod sum", "product sum"}
_MS_NAMES = {"ms", "minimum_sum", "min_sum", "1", "minimum sum", "min sum",
             "msl", "minimum_sum_log", "ms_log", "min_sum_log", "3", "minimum sum_log", "minimum sum log"}
_PSL_NAMES = {"ps_log", "product_sum_log", "prod_sum_log", "2", "psl"}


def parse_bp_method(method) -> int:
    """ldpc v1 bp_method names -> QD_*.  'ms' and 'msl' both mean min-sum in the
    log domain (ldpc v1 maps min_sum to its log variant)."""
    key = str(method).strip().lower()
    if key in _PS_NAMES:
        return _abi.QD_PRODUCT_SUM
    if key in _MS_NAMES:
        return _abi.QD_MIN_SUM
    if key in _PSL_NAMES:
        raise NotImplementedError("bp_method 'ps_log' (product-sum, log domain) is not implemented by this build; "
                                  "use 'ps' or 'ms'")
    raise ValueError(f"unknown bp_method {method!r}")


def parse_precision(precision) -> int:
    key = str(precision).lower()
    if key in ("f32", "fp32", "float32", "float"):
        return _abi.QD_F32
    if key in ("f64", "fp64", "float64", "double"):
        return _abi.QD_F64
    raise ValueError(f"unknown precision {precision!r}")


def as_csr01(H) -> sp.csr_matrix:
    """Any dense/sparse 0/1 matrix -> canonical CSR (sorted, deduplicated mod 2)."""
    if sp.issparse(H):
        M = sp.csr_matrix(H, dtype=np.int64)
    else:
        M = sp.csr_matrix(np.asarray(H, dtype=np.int64))
    M.sum_duplicates()
    M.data %= 2
    M.eliminate_zeros()
    M.sort_indices()
    M.data[:] = 1
    return M


class Decoder:
    def __init__(self, H, channel_probs, *, method="ms", precision="f32", max_iter: int = 0,
                 ms_scaling: float = 0.0, flip_sets=None, ssf: bool | None = None, ssf_max_steps: int = 0,
                 logicals=None, n_data: int | None = None, fold_blocks: int = 1, device: int = 0):
        self._lib = _abi.load()
        H = as_csr01(H)
        self.H = H
        self.m, self.n = H.shape
        self.n_data = self.n if n_data is None else int(n_data)
        self.fold_blocks = int(fold_blocks)
        self.device = int(device)
        self._handle = C.c_void_p()
        rp = np.ascontiguousarray(H.indptr, dtype=np.int32)
        ci = np.ascontiguousarray(H.indices, dtype=np.int32)
        _abi.check(self._lib.qd_graph_create(self.m, self.n, _abi.ptr(rp), _abi.ptr(ci), self.n_data,
                                             self.fold_blocks, self.device, C.byref(self._handle)),
                   "qd_graph_create")
        for name, value in DEFAULT_OPTIONS.items():
            self.set_option(name, value)
        self.method = parse_bp_method(method)
        self.precision = parse_precision(precision)
        self.max_iter = int(max_iter)
        self.ms_scaling = float(ms_scaling)
        self.ssf_max_steps = int(ssf_max_steps)
        self.has_flip_sets = False
        if flip_sets is not None:
            self.set_flip_sets(flip_sets)
        self.ssf = bool(self.has_flip_sets if ssf is None else ssf)
        self.k = 0
        if logicals is not None:
            self.set_logicals(logicals)
        self.set_priors(channel_probs)

    # ------------------------------------------------------------ graph data
    def set_priors(self, channel_probs) -> None:
        p = np.ascontiguousarray(np.broadcast_to(np.asarray(channel_probs, dtype=np.float64), (self.n,)))
        self.channel_probs = p.copy()
        _abi.check(self._lib.qd_graph_set_priors(self._handle, _abi.ptr(p)), "qd_graph_set_priors")

    def set_flip_sets(self, generators) -> None:
        G = as_csr01(generators)
        if G.shape[1] != self.n:
            raise ValueError("flip-set generators must have one column per decoding column")
        gp = np.ascontiguousarray(G.indptr, dtype=np.int32)
        gi = np.ascontiguousarray(G.indices, dtype=np.int32)
        _abi.check(self._lib.qd_graph_set_flipsets(self._handle, G.shape[0], _abi.ptr(gp), _abi.ptr(gi)),
                   "qd_graph_set_flipsets")
        self.has_flip_sets = True

    def set_logicals(self, lz) -> None:
        """Logical operators (k x n_data, dense or scipy sparse) for the fused
        failure check; handed over as CSR supports (qd_graph_set_logicals_csr),
        so codes with thousands of sparse logicals never build a dense k x n
        array."""
        if not sp.issparse(lz) and np.ndim(lz) != 2:  # csr_matrix would read a 1-D array as one row
            raise ValueError("logicals must be k x n_data")
        L = sp.csr_matrix(lz, copy=True) if sp.issparse(lz) else sp.csr_matrix(np.asarray(lz) % 2)
        if L.ndim != 2 or L.shape[1] != self.n_data:
            raise ValueError("logicals must be k x n_data")
        L.sum_duplicates()
        L.data %= 2
        L.eliminate_zeros()
        L.sort_indices()
        ptr = np.ascontiguousarray(L.indptr, dtype=np.int32)
        idx = np.ascontiguousarray(L.indices, dtype=np.int32)
        _abi.check(self._lib.qd_graph_set_logicals_csr(self._handle, L.shape[0], _abi.ptr(ptr), _abi.ptr(idx)),
                   "qd_graph_set_logicals_csr")
        self.k = L.shape[0]

    def _params(self, syn_flags: int = 0, ssf: bool | None = None) -> _abi.QdParams:
        return _abi.QdParams(self.max_iter, self.method, self.precision,
                             int(self.ssf if ssf is None else ssf), self.ssf_max_steps, int(syn_flags),
                             self.ms_scaling)

    @property
    def llr_dtype(self):
        return np.float32 if self.precision == _abi.QD_F32 else np.float64

    # ------------------------------------------------------------ decoding
    def decode(self, syn=None, *, base=None, readout=None, syn_flags: int = 0, ssf: bool | None = None,
               want=("x", "corr", "iters", "status", "ssf_steps", "fail"), packed: bool = False) -> dict:
        """Decode B shots from host arrays; returns numpy arrays for `want`
        (any of x, corr, llr, iters, status, ssf_steps, fail).  packed=True:
        syn / base / readout are bit-packed rows (uint64 words, pack_rows;
        QD_INPUT_PACKED)."""
        def u8(a, cols):
            if a is None:
                return None
            if packed:
                return np.ascontiguousarray(np.asarray(a), dtype=np.uint64).reshape(-1, (cols + 63) // 64)
            a = np.ascontiguousarray(np.asarray(a), dtype=np.uint8)
            return a.reshape(-1, cols)
        if packed:
            syn_flags = int(syn_flags) | QD_INPUT_PACKED
        syn = u8(syn, self.m)
        base = u8(base, self.n_data)
        readout = u8(readout, self.n_data)
        B = next(a.shape[0] for a in (syn, base, readout) if a is not None)
        for a in (syn, base, readout):
            if a is not None and a.shape[0] != B:
                raise ValueError("inconsistent batch sizes")
        out = {}
        if "x" in want:
            out["x"] = np.empty((B, self.n), np.uint8)
        if "corr" in want:
            out["corr"] = np.empty((B, self.n_data), np.uint8)
        if "llr" in want:
            out["llr"] = np.empty((B, self.n), self.llr_dtype)
        if "iters" in want:
            out["iters"] = np.empty(B, np.int32)
        if "status" in want:
            out["status"] = np.empty(B, np.uint8)
        if "ssf_steps" in want:
            out["ssf_steps"] = np.empty(B, np.int32)
        if "fail" in want:
            out["fail"] = np.empty(B, np.uint8)
        prm = self._params(syn_flags, ssf)
        g = out.get
        _abi.check(self._lib.qd_decode_batch(
            self._handle, C.byref(prm), B, _abi.ptr(syn), _abi.ptr(base), _abi.ptr(readout),
            _abi.ptr(g("x")), _abi.ptr(g("corr")), _abi.ptr(g("llr")), _abi.ptr(g("iters")),
            _abi.ptr(g("status")), _abi.ptr(g("ssf_steps")), _abi.ptr(g("fail"))), "qd_decode_batch")
        return out

    def decode_device(self, B: int, *, syn=None, base=None, readout=None, x=None, corr=None, llr=None,
                      iters=None, status=None, ssf_steps=None, fail=None, syn_flags: int = 0,
                      ssf: bool | None = None, stream=None, packed: bool = False) -> None:
        """Enqueue a decode of B device-resident shots (torch tensors or raw
        device pointers) on `stream` (default: torch's current stream).
        packed=True: syn / base / readout are bit-packed rows, int64 tensors
        [B][ceil(m/64)] / [B][ceil(n_data/64)] (sample_storage_device(packed=True)
        writes them; QD_INPUT_PACKED)."""
        if stream is None:
            stream = _current_stream(self.device)
        B = int(B)
        llr_t = "float32" if self.precision == _abi.QD_F32 else "float64"
        in_t = "int64" if packed else "uint8"
        wcols = (lambda c: (c + 63) // 64) if packed else (lambda c: c)
        if packed:
            syn_flags = int(syn_flags) | QD_INPUT_PACKED
        for name, t, dt, cols in (("syn", syn, in_t, wcols(self.m)), ("base", base, in_t, wcols(self.n_data)),
                                  ("readout", readout, in_t, wcols(self.n_data)), ("x", x, "uint8", self.n),
                                  ("corr", corr, "uint8", self.n_data), ("llr", llr, llr_t, self.n),
                                  ("iters", iters, "int32", 1), ("status", status, "uint8", 1),
                                  ("ssf_steps", ssf_steps, "int32", 1), ("fail", fail, "uint8", 1)):
            self._check_device_buffer(name, t, dt, B * cols)
        prm = self._params(syn_flags, ssf)
        _abi.check(self._lib.qd_decode_batch_device(
            self._handle, C.byref(prm), int(B), _abi.ptr(syn), _abi.ptr(base), _abi.ptr(readout), _abi.ptr(x),
            _abi.ptr(corr), _abi.ptr(llr), _abi.ptr(iters), _abi.ptr(status), _abi.ptr(ssf_steps), _abi.ptr(fail),
            C.c_void_p(stream)), "qd_decode_batch_device")

    def _check_device_buffer(self, name, t, dtype: str, numel: int) -> None:
        """A torch tensor handed to a *_device call must be a contiguous tensor on
        this decoder's GPU with the ABI's element type and at least `numel`
        elements (raw integer pointers are passed through unchecked)."""
        if t is None or isinstance(t, int) or not hasattr(t, "data_ptr"):
            return
        if not t.is_cuda or t.device.index != self.device:
            raise ValueError(f"{name}: expected a tensor on cuda:{self.device}, got {t.device}")
        if str(t.dtype).rsplit(".", 1)[-1] != dtype:
            raise ValueError(f"{name}: expected dtype {dtype}, got {t.dtype}")
        if not t.is_contiguous():
            raise ValueError(f"{name}: tensor must be contiguous")
        if t.numel() < numel:
            raise ValueError(f"{name}: {t.numel()} elements, the batch needs {numel}")

    def sample_storage_device(self, rounds: int, p_data: float, p_meas: float, seed: int, stream_id: int,
                              shot0: int, B: int, syn, readout, stream=None, packed: bool = False) -> None:
        """Storage-experiment sampler (H must be the plain Hz graph).  packed=True
        writes bit-packed rows: syn int64 [B][ceil((rounds+1) m / 64)], readout
        int64 [B][ceil(n / 64)] (the same shots as the byte rows, pack_rows of them)."""
        if stream is None:
            stream = _current_stream(self.device)
        if packed:
            self._check_device_buffer("syn", syn, "int64", B * (((rounds + 1) * self.m + 63) // 64))
            self._check_device_buffer("readout", readout, "int64", B * ((self.n + 63) // 64))
            _abi.check(self._lib.qd_sample_storage_packed_device(
                self._handle, int(rounds), float(p_data), float(p_meas), int(seed) & 0xFFFFFFFF,
                int(stream_id) & 0xFFFFFFFF, int(shot0), int(B), _abi.ptr(syn), _abi.ptr(readout),
                C.c_void_p(stream)), "qd_sample_storage_packed_device")
            return
        _abi.check(self._lib.qd_sample_storage_device(
            self._handle, int(rounds), float(p_data), float(p_meas), int(seed) & 0xFFFFFFFF,
            int(stream_id) & 0xFFFFFFFF, int(shot0), int(B), _abi.ptr(syn), _abi.ptr(readout), C.c_void_p(stream)),
            "qd_sample_storage_device")

    # ------------------------------------------------------------ OSD on the device
    @property
    def osd_device_supported(self) -> bool:
        return bool(self._lib.qd_osd_device_supported(self._handle))

    def osd_device(self, B: int, *, llr, method: str = "osd_cs", order: int = 0, syn=None, syn_flags: int = 0,
                   status=None, base=None, readout=None, osd0=None, osdw=None, corr=None, fail=None,
                   stream=None) -> None:
        """Enqueue OSD (qd_osd_batch_device) for the shots whose `status` lacks
        the BP-converged bit, on device buffers; `llr` is the BP soft output
        (float32 or float64 tensor)."""
        from .osd import OSD_METHODS
        if method not in OSD_METHODS:
            raise ValueError(f"unknown OSD method {method!r}")
        if stream is None:
            stream = _current_stream(self.device)
        prec = _abi.QD_F32 if str(getattr(llr, "dtype", "")).endswith("float32") else _abi.QD_F64
        _abi.check(self._lib.qd_osd_batch_device(
            self._handle, OSD_METHODS[method], int(order), int(B), _abi.ptr(syn), int(syn_flags), _abi.ptr(llr), prec,
            _abi.ptr(status), _abi.ptr(base), _abi.ptr(readout), _abi.ptr(osd0), _abi.ptr(osdw), _abi.ptr(corr),
            _abi.ptr(fail), C.c_void_p(stream)), "qd_osd_batch_device")

    def set_wave_occupancy(self, waves_per_cu: int = 0) -> None:
        """Waves per CU of the wave BP kernels (qd_graph_set_wave_occupancy):
        0 = the default; more for decodes that run concurrently on several
        streams.  Results do not depend on it."""
        _abi.check(self._lib.qd_graph_set_wave_occupancy(self._handle, int(waves_per_cu)),
                   "qd_graph_set_wave_occupancy")

    def set_option(self, name: str, value) -> None:
        """Kernel choice of this handle (qd_graph_set_option): name in OPTIONS;
        for "ssf" the value may be a SSF_KERNELS name."""
        if name == "ssf" and isinstance(value, str):
            value = SSF_KERNELS[value]
        _abi.check(self._lib.qd_graph_set_option(self._handle, OPTIONS[name], int(value)), f"set_option({name})")

    def get_option(self, name: str) -> int:
        v = C.c_int32(0)
        _abi.check(self._lib.qd_graph_get_option(self._handle, OPTIONS[name], C.byref(v)), f"get_option({name})")
        return v.value

    def ssf_tables(self) -> tuple[bool, int]:
        """(the graph qualifies for the table-driven SSF kernel, its table bytes)."""
        has, nb = C.c_int32(0), C.c_int64(0)
        _abi.check(self._lib.qd_graph_ssf_tables(self._handle, C.byref(has), C.byref(nb)), "qd_graph_ssf_tables")
        return bool(has.value), int(nb.value)

    def set_ssf_stream(self, stream) -> None:
        """Run the SSF kernel of later decode_device calls on `stream` (a torch
        stream or a raw hipStream_t; None = the decode's own stream); see
        qd_graph_set_ssf_stream: the caller synchronises with that stream.
        Split decodes alternate between two SSF queues, so this handle's next
        decode (triage + BP) overlaps this one's SSF kernel; the one after it
        waits for it."""
        raw = None if stream is None else int(getattr(stream, "cuda_stream", stream))
        _abi.check(self._lib.qd_graph_set_ssf_stream(self._handle, C.c_void_p(raw)), "qd_graph_set_ssf_stream")

    # ------------------------------------------------------------ timing
    def set_timing(self, capacity: int) -> None:
        """Record HIP events around the BP and SSF kernels of the next
        `capacity` decode calls (on their launch stream)."""
        _abi.check(self._lib.qd_graph_set_timing(self._handle, int(capacity)), "qd_graph_set_timing")
        self._t_cap = int(capacity)

    def read_timing(self):
        """(bp_ms[calls], ssf_ms[calls]) of the recorded calls; resets the ring."""
        cap = getattr(self, "_t_cap", 0)
        bp = np.zeros(max(cap, 1), np.float32)
        ssf = np.zeros(max(cap, 1), np.float32)
        cnt = C.c_int32(0)
        _abi.check(self._lib.qd_graph_read_timing(self._handle, _abi.ptr(bp), _abi.ptr(ssf), cap, C.byref(cnt)),
                   "qd_graph_read_timing")
        return bp[:cnt.value].astype(np.float64), ssf[:cnt.value].astype(np.float64)

    def read_timing_detail(self):
        """(pre_ms, bp_ms, ssf_ms, listed) per recorded call: the BP stage's
        pre-pass (shot triage), the BP kernel alone, the SSF kernel, and the
        shots the triage left to the BP kernel (-1: no two-pass launch);
        resets the ring."""
        cap = getattr(self, "_t_cap", 0)
        pre, bp, ssf = (np.zeros(max(cap, 1), np.float32) for _ in range(3))
        listed = np.zeros(max(cap, 1), np.int64)
        cnt = C.c_int32(0)
        _abi.check(self._lib.qd_graph_read_timing_detail(self._handle, _abi.ptr(pre), _abi.ptr(bp), _abi.ptr(ssf),
                                                         _abi.ptr(listed), cap, C.byref(cnt)),
                   "qd_graph_read_timing_detail")
        n = cnt.value
        return pre[:n].astype(np.float64), bp[:n].astype(np.float64), ssf[:n].astype(np.float64), listed[:n]

    def last_kernels(self) -> tuple[str, str, str]:
        """(BP kernel, SSF kernel, pre-pass) the last decode call launched, in
        rocprofv3's spelling with template arguments ("" for a stage that did
        not run); the pre-pass (lean launches' shot triage) runs inside the BP
        timing."""
        bp, ssf, pre = (C.create_string_buffer(512) for _ in range(3))
        _abi.check(self._lib.qd_graph_last_kernels(self._handle, bp, 512, ssf, 512, pre, 512),
                   "qd_graph_last_kernels")
        return bp.value.decode(), ssf.value.decode(), pre.value.decode()

    def close(self) -> None:
        if getattr(self, "_handle", None) and self._handle.value:
            self._lib.qd_graph_destroy(self._handle)
            self._handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


QD_INPUT_PACKED = _abi.QD_INPUT_PACKED  # qd_syn_flags: bit-packed input rows


def pack_rows(bits) -> np.ndarray:
    """Bit-pack 0/1 rows (uint8 [B][L]) into the QD_INPUT_PACKED layout: uint64
    [B][ceil(L/64)], bit j of word w = element 64 w + j (little-endian: byte for
    byte Stim's bit_packed=True rows, zero-padded to 8 bytes)."""
    a = np.asarray(bits, dtype=np.uint8) & 1
    a = a.reshape(a.shape[0], -1) if a.ndim > 1 else a.reshape(1, -1)
    B, L = a.shape
    W = (L + 63) // 64
    by = np.packbits(a, axis=1, bitorder="little")
    out = np.zeros((B, W * 8), np.uint8)
    out[:, :by.shape[1]] = by
    return out.view("<u8").reshape(B, W).astype(np.uint64)


def unpack_rows(words, length: int) -> np.ndarray:
    """Inverse of pack_rows: uint8 [B][length]."""
    w = np.ascontiguousarray(np.asarray(words).astype("<u8"))
    B = w.shape[0] if w.ndim > 1 else 1
    by = w.reshape(B, -1).view(np.uint8)
    return np.unpackbits(by, axis=1, bitorder="little")[:, :length].astype(np.uint8)


def count_flags_device(flags, B: int, mask: int, out, stream=None, device: int = 0) -> None:
    """out (device int64[1]) += #{b : flags[b] & mask}."""
    lib = _abi.load()
    if stream is None:
        stream = _current_stream(device)
    _abi.check(lib.qd_count_flags_device(_abi.ptr(flags), int(B), int(mask) & 0xFF, _abi.ptr(out),
                                         C.c_void_p(stream)), "qd_count_flags_device")


def _current_stream(device: int) -> int:
    if _abi.torch is not None and _abi.torch.cuda.is_available():
        return int(_abi.torch.cuda.current_stream(device).cuda_stream)
    return 0
