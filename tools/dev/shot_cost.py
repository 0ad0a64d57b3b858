"""Dev: per-launch BP kernel time at low p under output variants (which per-shot
work costs what).  Run on the GPU box."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from exp_ldpc_amd.decoder import Decoder
import bench
code = bench.load_code()
hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
B = 1 << 18
dev = torch.device("cuda", 0)
for p in (0.001, 0.03):
    dec = Decoder(hz, 2 * p / 3, method="ms", precision="f32", max_iter=50, flip_sets=hx, logicals=lz)
    syn = torch.empty((B, 108), dtype=torch.uint8, device=dev)
    rd = torch.empty((B, 225), dtype=torch.uint8, device=dev)
    dec.sample_storage_device(0, p, p, 1, 0, 0, B, syn, rd)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    status = torch.empty(B, dtype=torch.uint8, device=dev)
    fail = torch.empty(B, dtype=torch.uint8, device=dev)
    variants = {
        "full": dict(syn=syn, readout=rd, iters=iters, status=status, fail=fail),
        "no_fail": dict(syn=syn, iters=iters, status=status),
        "iters_only": dict(syn=syn, iters=iters),
        "nothing": dict(syn=syn),
        "zero_syn": dict(iters=iters),
    }
    for name, kw in variants.items():
        for ssf in (True, False):
            dec.decode_device(B, ssf=ssf, **kw)
            torch.cuda.synchronize()
            dec.set_timing(5)
            for _ in range(5):
                dec.decode_device(B, ssf=ssf, **kw)
            bp, sf = dec.read_timing()
            print(f"p={p} {name:10s} ssf={int(ssf)} bp_ms={bp.mean():.3f} ssf_ms={sf.mean():.3f}", flush=True)
