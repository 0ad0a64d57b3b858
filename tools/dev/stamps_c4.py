"""Dev: phase timers of bp_ms_lds64_kernel on config 4 (needs libqdec_hip_stamps.so,
`python -m exp_ldpc_amd.build --stamps`).  Prints s_memtime ticks per shot for
the shot phases (S = syndrome + state image, D = variable pass, B = syndrome
test + reset, Q = queue stores, top = next-shot hand-out) and per iteration.

Usage: python tools/dev/stamps_c4.py [p ...]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("QDEC_LIB", os.path.join(ROOT, "exp_ldpc_amd", "libqdec_hip_stamps.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import torch  # noqa: E402

from exp_ldpc_amd import _abi  # noqa: E402
from exp_ldpc_amd.decoder import Decoder  # noqa: E402

lib = _abi.load()
lib.qd_dev_read_stamps_block.argtypes = [C.c_void_p, C.c_int, C.c_int]


def csr(path, key):
    d = np.load(os.path.join(ROOT, "tests", "golden", path))
    return sp.csr_matrix((np.ones(d[key + "_indices"].size, np.uint8), d[key + "_indices"], d[key + "_indptr"]),
                         shape=tuple(d[key + "_shape"]))


hz, hx = csr("hgp_80_3_4_s2025_checks.npz", "hz"), csr("hgp_80_3_4_s2025_checks.npz", "hx")
lz = csr("hgp_80_3_4_s2025_logicals.npz", "lz")
m, n = hz.shape
dev = torch.device("cuda", 0)
B = 1 << 17
names = ["S", "D", "B", "Q", "top"]
for p in [float(x) for x in (sys.argv[1:] or ["0.005", "0.03"])]:
    sampler = Decoder(hz, 2 * p / 3, method="ms", precision="f32", max_iter=50, device=0)
    syn = torch.empty((B, m), dtype=torch.uint8, device=dev)
    rd = torch.empty((B, n), dtype=torch.uint8, device=dev)
    sampler.sample_storage_device(0, p, p, 1, 200, 0, B, syn, rd)
    dec = Decoder(hz, 2 * p / 3, method="ms", precision="f64", max_iter=50, flip_sets=hx, logicals=lz, device=0)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    status = torch.empty(B, dtype=torch.uint8, device=dev)
    fail = torch.empty(B, dtype=torch.uint8, device=dev)
    buf = np.zeros(64, np.uint64)
    for rep in range(2):
        lib.qd_dev_read_stamps_block(buf.ctypes.data, 64, 1)
        dec.decode_device(B, syn=syn, readout=rd, iters=iters, status=status, fail=fail)
        torch.cuda.synchronize()
    lib.qd_dev_read_stamps_block(buf.ctypes.data, 64, 1)
    st = buf[16:32].astype(np.float64)
    waves = 1024 // 64
    shots = st[8] / waves
    its = st[9] / waves
    print(f"p={p} kernel={dec.last_kernels()[0]} shots={shots:.0f} iters/shot={its / shots:.2f} "
          "ticks/shot (per wave): " + " ".join(f"{nm}={st[i] / waves / shots:.0f}" for i, nm in enumerate(names)) +
          f" | D/iter={st[1] / waves / its:.0f} B/iter={st[2] / waves / its:.0f}")
