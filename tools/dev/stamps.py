"""Dev: phase timers of the min-sum kernel (needs libqdec_hip_stamps.so)."""
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
names = ["wait_syn", "stage+init", "iterations", "post", "finalize", "loop_top"]
for p in [float(x) for x in (sys.argv[1:] or ["0.001", "0.1"])]:
    dec = Decoder(hz, 2 * p / 3, method="ms", precision=os.environ.get("STAMP_PREC", "f32"), max_iter=50, flip_sets=hx, logicals=lz)
    syn = torch.empty((B, 108), dtype=torch.uint8, device=dev)
    rd = torch.empty((B, 225), dtype=torch.uint8, device=dev)
    dec.sample_storage_device(0, p, p, 1, 0, 0, B, syn, rd)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    status = torch.empty(B, dtype=torch.uint8, device=dev)
    fail = torch.empty(B, dtype=torch.uint8, device=dev)
    for label, kw in (("full", dict(syn=syn, readout=rd, iters=iters, status=status, fail=fail)),
                      ("no_fail", dict(syn=syn, iters=iters, status=status))):
        for ssf in (True, False):
            dec.decode_device(B, ssf=ssf, **kw)
            torch.cuda.synchronize()
            buf = np.zeros(64, np.uint64)
            lib.qd_dev_read_stamps(buf.ctypes.data, 64, 1)
            dec.decode_device(B, ssf=ssf, **kw)
            torch.cuda.synchronize()
            lib.qd_dev_read_stamps(buf.ctypes.data, 64, 1)
            shots = int(buf[9]); its = int(buf[8])
            if not shots:  # the compact path's kernels stamp other slots (stamps_cmp.py)
                continue
            print(f"p={p} {label} ssf={int(ssf)} shots={shots} iters/shot={its/shots:.2f} cycles/shot: " +
                  " ".join(f"{n}={buf[i]/shots:.0f}" for i, n in enumerate(names)) +
                  f" | per-iter={buf[2]/its:.0f} | waves={int(buf[12])} ticks/wave={buf[10]/max(1,buf[12]):.0f}"
                  f" real_us/wave={buf[11]/max(1,buf[12])/100:.1f}", flush=True)

# SSF kernel phases (slots 16..31)
for p in [float(x) for x in (sys.argv[1:] or ["0.001", "0.1"])]:
    dec = Decoder(hz, 2 * p / 3, method="ms", precision=os.environ.get("STAMP_PREC", "f32"), max_iter=50, flip_sets=hx, logicals=lz)
    syn = torch.empty((B, 108), dtype=torch.uint8, device=dev)
    rd = torch.empty((B, 225), dtype=torch.uint8, device=dev)
    dec.sample_storage_device(0, p, p, 1, 0, 0, B, syn, rd)
    fail = torch.empty(B, dtype=torch.uint8, device=dev)
    dec.decode_device(B, syn=syn, readout=rd, fail=fail)
    torch.cuda.synchronize()
    buf = np.zeros(64, np.uint64)
    lib.qd_dev_read_stamps(buf.ctypes.data, 64, 1)
    dec.decode_device(B, syn=syn, readout=rd, fail=fail)
    torch.cuda.synchronize()
    lib.qd_dev_read_stamps(buf.ctypes.data, 64, 1)
    b = buf[16:32]
    shots, steps = int(b[7]), int(b[6])
    if shots:
        print(f"SSF p={p} shots={shots} steps/shot={steps/shots:.2f} listed/step={b[5]/max(1,steps):.1f} per-step ticks: "
              f"gather+compact={b[0]/steps:.0f} score={b[1]/steps:.0f} select={b[2]/steps:.0f} apply={b[3]/steps:.0f} | "
              f"per-shot: load={b[12]/shots:.0f} tail={b[13]/shots:.0f} fin_words={b[8]/shots:.0f} "
              f"fin_logicals={b[9]/shots:.0f} fin_stores={b[14]/shots:.0f}", flush=True)
