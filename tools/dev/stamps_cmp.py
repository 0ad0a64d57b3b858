"""Dev: phase timers of the two-pass lean path's BP kernel (bp_ms_cmp_kernel,
stamp slots 32..47; needs libqdec_hip_stamps.so: python -m exp_ldpc_amd.build --stamps)."""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("QDEC_LIB", os.path.join(ROOT, "exp_ldpc_amd", "libqdec_hip_stamps.so"))
sys.path.insert(0, ROOT)
import numpy as np, torch
from exp_ldpc_amd import _abi
from exp_ldpc_amd.decoder import Decoder
import bench
lib = _abi.load()
lib.qd_dev_read_stamps.argtypes = [C.c_void_p, C.c_int, C.c_int]
code = bench.load_code()
hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
B = 1 << 18
dev = torch.device("cuda", 0)
names = ["entry+init", "iterations", "epilogue", "chunk", "prologue"]
for p in [float(x) for x in (sys.argv[1:] or ["0.001", "0.01", "0.1"])]:
    dec = Decoder(hz, 2 * p / 3, method="ms", precision=os.environ.get("STAMP_PREC", "f64"), max_iter=50,
                  flip_sets=hx, logicals=lz)
    syn = torch.empty((B, 108), dtype=torch.uint8, device=dev)
    rd = torch.empty((B, 225), dtype=torch.uint8, device=dev)
    dec.sample_storage_device(0, p, p, 1, 0, 0, B, syn, rd)
    out = dict(iters=torch.empty(B, dtype=torch.int32, device=dev), status=torch.empty(B, dtype=torch.uint8, device=dev),
               ssf_steps=torch.empty(B, dtype=torch.int32, device=dev), fail=torch.empty(B, dtype=torch.uint8, device=dev))
    buf = np.zeros(64, np.uint64)
    for rep in range(2):
        dec.decode_device(B, syn=syn, readout=rd, **out)
        torch.cuda.synchronize()
        lib.qd_dev_read_stamps(buf.ctypes.data, 64, 1)
    b = buf[32:48]
    shots, its, waves = int(b[9]), int(b[8]), int(max(1, b[12]))
    print(f"p={p} listed={shots} iters/listed={its / max(1, shots):.2f} cycles per listed shot: " +
          " ".join(f"{n}={b[i] / max(1, shots):.0f}" for i, n in enumerate(names)) +
          f" | per-iter={b[1] / max(1, its):.0f} | waves={waves} ticks/wave={b[10] / waves:.0f} "
          f"prologue/wave={b[4] / waves:.0f}", flush=True)
