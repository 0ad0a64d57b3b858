"""Dev: SSF kernel time per launch at several p (library events)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from exp_ldpc_amd.decoder import Decoder
import bench
code = bench.load_code()
hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
B = 1 << 18
dev = torch.device("cuda", 0)
tag = os.environ.get("QDEC_LIB", "default").split("/")[-1]
for p in (0.01, 0.03, 0.1):
    dec = Decoder(hz, 2 * p / 3, method="ms", precision="f32", max_iter=50, flip_sets=hx, logicals=lz)
    syn = torch.empty((B, 108), dtype=torch.uint8, device=dev)
    rd = torch.empty((B, 225), dtype=torch.uint8, device=dev)
    dec.sample_storage_device(0, p, p, 1, 0, 0, B, syn, rd)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    status = torch.empty(B, dtype=torch.uint8, device=dev)
    fail = torch.empty(B, dtype=torch.uint8, device=dev)
    ss = torch.empty(B, dtype=torch.int32, device=dev)
    kw = dict(syn=syn, readout=rd, iters=iters, status=status, fail=fail, ssf_steps=ss)
    dec.decode_device(B, **kw)
    torch.cuda.synchronize()
    dec.set_timing(5)
    for _ in range(5):
        dec.decode_device(B, **kw)
    bp, sf = dec.read_timing()
    print(f"{tag} p={p} bp_ms={bp.mean():.3f} ssf_ms={sf.mean():.3f} fails={int(fail.sum())}", flush=True)
