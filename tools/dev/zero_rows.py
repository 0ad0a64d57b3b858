"""Dev: how often the f64 LEAN min-sum kernel meets a check row holding an exact
zero message (the rare path of QDEC_MS_SIGNBIT).  Needs libqdec_hip_stamps.so."""
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
for p in [float(x) for x in (sys.argv[1:] or ["0.001", "0.01", "0.0316228", "0.1"])]:
    dec = Decoder(hz, 2 * p / 3, method="ms", precision="f64", max_iter=50, flip_sets=hx, logicals=lz)
    syn = torch.empty((B, 108), dtype=torch.uint8, device=dev)
    rd = torch.empty((B, 225), dtype=torch.uint8, device=dev)
    dec.sample_storage_device(0, p, p, 1, 0, 0, B, syn, rd)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    status = torch.empty(B, dtype=torch.uint8, device=dev)
    fail = torch.empty(B, dtype=torch.uint8, device=dev)
    buf = np.zeros(64, np.uint64)
    dec.decode_device(B, syn=syn, readout=rd, iters=iters, status=status, fail=fail)
    torch.cuda.synchronize()
    lib.qd_dev_read_stamps(buf.ctypes.data, 64, 1)
    dec.decode_device(B, syn=syn, readout=rd, iters=iters, status=status, fail=fail)
    torch.cuda.synchronize()
    lib.qd_dev_read_stamps(buf.ctypes.data, 64, 1)
    its = int(buf[8])
    print(f"p={p} shot-iterations={its} zero-row wave-iterations={int(buf[13])} ({buf[13]/max(1,its):.2e}) "
          f"zero-row lanes={int(buf[14])}", flush=True)
