"""Dev: time the f64 lean BP launch (bench.py's call, two-pass path) at given p
on 2^18 device-sampled shots with whatever library QDEC_LIB names (diagnostic
builds: tools/dev/diag_conflicts.sh).  Prints per p the BP kernel's HIP-event
time (3 timed launches) and the mean iterations."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from exp_ldpc_amd.decoder import Decoder  # noqa: E402

code = bench.load_code()
hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
m, n = hz.shape
B = 1 << 18
dev = torch.device("cuda", 0)
for p in [float(a) for a in (sys.argv[1:] or ["0.1"])]:
    dec = Decoder(hz, 2 * p / 3, method="ms", precision="f64", max_iter=50, ms_scaling=0.0, flip_sets=hx, logicals=lz)
    sw = torch.empty((B, (m + 63) // 64), dtype=torch.int64, device=dev)
    rw = torch.empty((B, (n + 63) // 64), dtype=torch.int64, device=dev)
    dec.sample_storage_device(0, p, p, bench.SEED, 8, 0, B, sw, rw, packed=True)
    out = {k: torch.empty(B, dtype=dt, device=dev) for k, dt in
           (("iters", torch.int32), ("status", torch.uint8), ("ssf_steps", torch.int32), ("fail", torch.uint8))}
    dec.decode_device(B, syn=sw, readout=rw, packed=True, **out)
    torch.cuda.synchronize()
    dec.set_timing(3)
    for _ in range(3):
        dec.decode_device(B, syn=sw, readout=rw, packed=True, **out)
    torch.cuda.synchronize()
    pre, bp, ssf, listed = dec.read_timing_detail()
    it = out["iters"].to(torch.float64).mean().item()
    print(f"p={p} bp_ms={np.round(bp, 3).tolist()} mean_iters={it:.2f} kernel={dec.last_kernels()[0]}", flush=True)
