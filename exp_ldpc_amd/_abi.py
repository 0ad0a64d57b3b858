"""ctypes binding of libqdec_hip.so (include/qdec.h).

The product path has no CPU fallback: if the HIP library is missing or cannot
be loaded this module raises, and every decoder constructor fails loudly.

torch (when importable) is imported *before* the library is loaded: the PyTorch
wheel bundles its own libamdhip64.so.7, and loading it first makes our library
bind to the same HIP runtime instead of a second copy from /opt/rocm.
"""
from __future__ import annotations

import ctypes as C
import os
import re

try:  # share torch's HIP runtime when torch is present (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the ABI itself
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QDEC_LIB") or os.path.join(HERE, "libqdec_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "qdec.h")

QD_PRODUCT_SUM, QD_MIN_SUM = 0, 1
QD_F64, QD_F32 = 0, 1
QD_SYN_ADD_BASE, QD_SYN_ADD_READOUT = 1, 2
QD_INPUT_PACKED = 16  # bit-packed input rows (include/qdec.h)
QD_ST_BP_CONVERGED, QD_ST_SATISFIED = 1, 2


class QdParams(C.Structure):
    _fields_ = [
        ("max_iter", C.c_int32),
        ("method", C.c_int32),
        ("precision", C.c_int32),
        ("ssf", C.c_int32),
        ("ssf_max_steps", C.c_int32),
        ("syn_flags", C.c_int32),
        ("ms_scaling", C.c_double),
    ]


class QdecError(RuntimeError):
    """A failed library call; rc is its status (<= -100: a HIP error)."""

    def __init__(self, msg: str, rc: int = 0):
        super().__init__(msg)
        self.rc = rc


_p = C.c_void_p
_i32 = C.c_int32
_i64 = C.c_int64
_u32 = C.c_uint32

# name -> (restype, argtypes)
SIGNATURES = {
    "qd_abi_version": (_i32, []),
    "qd_device_count": (_i32, []),
    "qd_last_error": (C.c_char_p, []),
    "qd_graph_create": (_i32, [_i32, _i32, _p, _p, _i32, _i32, _i32, C.POINTER(_p)]),
    "qd_graph_destroy": (_i32, [_p]),
    "qd_graph_create_host": (_i32, [_i32, _i32, _p, _p, _i32, _i32, C.POINTER(_p)]),
    "qd_graph_table_digest": (_i32, [_p, C.POINTER(C.c_uint64), C.POINTER(_i64)]),
    "qd_graph_set_flipsets": (_i32, [_p, _i32, _p, _p]),
    "qd_graph_set_logicals": (_i32, [_p, _i32, _p]),
    "qd_graph_set_logicals_csr": (_i32, [_p, _i32, _p, _p]),
    "qd_graph_set_priors": (_i32, [_p, _p]),
    "qd_decode_batch": (_i32, [_p, C.POINTER(QdParams), _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "qd_decode_batch_device": (_i32, [_p, C.POINTER(QdParams), _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "qd_sample_storage_device": (_i32, [_p, _i32, C.c_double, C.c_double, _u32, _u32, _i64, _i64, _p, _p, _p]),
    "qd_sample_storage_packed_device": (_i32, [_p, _i32, C.c_double, C.c_double, _u32, _u32, _i64, _i64, _p, _p,
                                               _p]),
    "qd_count_flags_device": (_i32, [_p, _i64, C.c_uint8, _p, _p]),
    "qd_osd_batch": (_i32, [_i32, _i32, _p, _p, _i32, _i32, _i64, _p, _p, _p, _p, _i32]),
    "qd_osd_last_error": (C.c_char_p, []),
    "qd_graph_set_timing": (_i32, [_p, _i32]),
    "qd_graph_set_ssf_stream": (_i32, [_p, _p]),
    "qd_graph_set_wave_occupancy": (_i32, [_p, _i32]),
    "qd_graph_read_timing": (_i32, [_p, _p, _p, _i32, C.POINTER(_i32)]),
    "qd_graph_read_timing_detail": (_i32, [_p, _p, _p, _p, _p, _i32, C.POINTER(_i32)]),
    "qd_graph_last_kernels": (_i32, [_p, C.c_char_p, _i32, C.c_char_p, _i32, C.c_char_p, _i32]),
    "qd_osd_device_supported": (_i32, [_p]),
    "qd_osd_batch_device": (_i32, [_p, _i32, _i32, _i64, _p, _i32, _p, _i32, _p, _p, _p, _p, _p, _p, _p, _p]),
    "qd_graph_set_option": (_i32, [_p, _i32, _i32]),
    "qd_graph_get_option": (_i32, [_p, _i32, C.POINTER(_i32)]),
    "qd_graph_ssf_tables": (_i32, [_p, C.POINTER(_i32), C.POINTER(_i64)]),
    "qd_graph_ssf_tables_copy": (_i32, [_p, _p, _p, _p, _p, C.POINTER(_i32), C.POINTER(_i32)]),
    "qd_graph_queue_layout": (_i32, [_p, _i64, _p]),
    "qd_graph_it1_tables_copy": (_i32, [_p, _i32, _p, _p, C.POINTER(_i32)]),
    "qd_graph_lds64_slots_copy": (_i32, [_p, _p, _p]),
    "qd_graph_hgp_info": (_i32, [_p, _p]),
    "qd_graph_hgp_set_slots": (_i32, [_p, _i32]),
    "qd_graph_hgp_source": (_i64, [_p, C.c_char_p, _i64]),
    "qd_graph_hgp_compile": (_i32, [_p]),
    "qd_graph_hgp_decode_bp": (_i32, [_p, _i64, _p, _p, _p, _p, _i32, C.c_double, _p]),
    "qd_gf2_rref": (_i64, [_p, _i64, _i64, _i64, _p, _i32]),
    "qd_gf2_extend_basis": (_i64, [_p, _i64, _p, _p, _i64, _i64, _i64, _p, _i64]),
}

# exported only by development builds (-DQDEC_DEV_HOOKS; not declared in include/qdec.h)
DEV_SIGNATURES = {
    "qd_graph_hgp_replace_source": (_i32, [_p, C.c_char_p]),
}


def header_symbols(path: str = HEADER) -> list[str]:
    """Every function the public header declares (used by the export test)."""
    text = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(qd_\w+)\s*\(", text, flags=re.M)))


_LIB = None


def load(path: str | None = None) -> C.CDLL:
    """Load (once) and type the HIP library; raises if it is absent."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise QdecError(f"{p} not found: build it with `python -m exp_ldpc_amd.build` (hipcc, gfx950). "
                        "There is no CPU fallback for the decoder.")
    lib = C.CDLL(p)
    for name, (res, args) in list(SIGNATURES.items()) + list(DEV_SIGNATURES.items()):
        fn = getattr(lib, name, None)
        if fn is None and name in DEV_SIGNATURES:
            continue  # development hooks exist only in QDEC_DEV_HOOKS builds
        fn.restype = res
        fn.argtypes = args
    if lib.qd_abi_version() != 1:
        raise QdecError("libqdec_hip.so ABI version mismatch")
    if path is None:
        _LIB = lib
    return lib


def check(rc: int, what: str = "qdec call") -> None:
    if rc != 0:
        msg = load().qd_last_error()
        raise QdecError(f"{what} failed ({rc}): {msg.decode() if msg else ''}", rc)


def ptr(a) -> C.c_void_p | None:
    """Raw pointer of a numpy array or torch tensor (None passes through).  The
    C ABI takes dense row-major buffers, so a strided view (e.g. a transposed
    array) is rejected instead of being read in the wrong order."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        if not a.is_contiguous():
            raise ValueError("qdec: tensor arguments must be contiguous (call .contiguous())")
        return C.c_void_p(a.data_ptr())
    if isinstance(a, C.c_void_p) or isinstance(a, int):
        return C.c_void_p(a) if isinstance(a, int) else a
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("qdec: array arguments must be C-contiguous (np.ascontiguousarray)")
    return a.ctypes.data_as(C.c_void_p)
