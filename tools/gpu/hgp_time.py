"""HGP kernel vs the generic lean f64 path, BP only (diagnostics):
python tools/gpu/hgp_time.py [slots ...]"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import torch  # noqa: E402

from exp_ldpc_amd import _abi  # noqa: E402
from exp_ldpc_amd.codes import read_quantum_code  # noqa: E402
from exp_ldpc_amd.decoder import Decoder  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
code = read_quantum_code(open(os.path.join(REPO, "tests", "golden", "hgp_12_3_4_s1234.qecc")))
hz = sp.csr_matrix(code.checks.z)
B = 1 << 18
slots = [int(a) for a in sys.argv[1:]] or [0]
out = []
strm = torch.cuda.Stream()
torch.cuda.set_stream(strm)  # events, generic decodes and HGP launches on one stream (not the null stream)
for p in (0.1, 0.056, 0.032, 0.01):
    dec = Decoder(hz, 2 * p / 3, method="ms", precision="f64", max_iter=50, device=0)
    syn = torch.empty((B, hz.shape[0]), dtype=torch.uint8, device="cuda:0")
    rd = torch.empty((B, hz.shape[1]), dtype=torch.uint8, device="cuda:0")
    dec.sample_storage_device(0, p, p, 1234, 0, 0, B, syn, rd)
    it_g = torch.empty(B, dtype=torch.int32, device="cuda:0")
    st_g = torch.empty(B, dtype=torch.uint8, device="cuda:0")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(2):
        dec.decode_device(B, syn=syn, iters=it_g, status=st_g)
    torch.cuda.synchronize()
    ev[0].record()
    dec.decode_device(B, syn=syn, iters=it_g, status=st_g)
    ev[1].record()
    torch.cuda.synchronize()
    gen_ms = ev[0].elapsed_time(ev[1])
    line = {"p": p, "generic_ms": gen_ms, "mean_iters": float(it_g.float().mean())}
    it_h = torch.empty(B, dtype=torch.int32, device="cuda:0")
    st_h = torch.empty(B, dtype=torch.uint8, device="cuda:0")
    for S in slots:
        _abi.check(dec._lib.qd_graph_hgp_set_slots(dec._handle, S), "slots")
        for _ in range(2):
            _abi.check(dec._lib.qd_graph_hgp_decode_bp(dec._handle, B, syn.data_ptr(), None, it_h.data_ptr(),
                                                       st_h.data_ptr(), 50, 0.0, C.c_void_p(torch.cuda.current_stream().cuda_stream)), "hgp")
        torch.cuda.synchronize()
        ev[0].record()
        _abi.check(dec._lib.qd_graph_hgp_decode_bp(dec._handle, B, syn.data_ptr(), None, it_h.data_ptr(),
                                                   st_h.data_ptr(), 50, 0.0, C.c_void_p(torch.cuda.current_stream().cuda_stream)), "hgp")
        ev[1].record()
        torch.cuda.synchronize()
        info = (C.c_int32 * 8)()
        dec._lib.qd_graph_hgp_info(dec._handle, info)
        line[f"hgp_ms_S{S}"] = ev[0].elapsed_time(ev[1])
        line[f"info_S{S}"] = list(info)
        line[f"iters_equal_S{S}"] = bool(torch.equal(it_h, it_g))
    print(json.dumps(line), flush=True)
    out.append(line)
if len(sys.argv) > 0:
    json.dump(out, open(os.path.join(REPO, "gpurun_out", "hgp_time.json"), "w"))
