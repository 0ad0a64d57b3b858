"""Debug the HGP kernel on the GPU with device printf in an edited source.

Needs the development build (qd_graph_hgp_replace_source):
  python -m exp_ldpc_amd.build --tag dev -DQDEC_DEV_HOOKS
  QDEC_LIB=exp_ldpc_amd/libqdec_hip_dev.so python tools/gpu/hgp_debug.py"""
import ctypes as C
import os
import sys

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
rng = np.random.default_rng(1)
B, p = 2, 0.01
e = (rng.random((B, 225)) < p).astype(np.uint8)
syn = ((hz @ e.T).T % 2).astype(np.uint8)
dec = Decoder(hz, 2 * p / 3, method="ms", precision="f64", max_iter=1, device=0)
L = dec._lib.qd_graph_hgp_source(dec._handle, None, 0)
buf = C.create_string_buffer(L + 1)
dec._lib.qd_graph_hgp_source(dec._handle, buf, L + 1)
src = buf.value.decode()
src = src.replace("    if (live) start();\n    int step = 0;",
                  "    if (live) start();\n    if (shot == 0 && ix == 5) printf(\"side %d ix %d s %d live %d pri0 %g v0 %g sb %x a.B %lld ms %g mi %d syn %p\\n\", SIDE, ix, s, (int)live, pri[0], v[0], sb, a.B, a.ms_scaling, a.max_iter, a.syn);\n    int step = 0;")
src = src.replace("                    s1[c] = with_sign(M1, par);",
                  "                    s1[c] = with_sign(M1, par);\n                    if (shot == 0 && SIDE == 0 && ix == 5) printf(\"chk %d pm %g %g po %g %g alpha %g\\n\", c, pm.x, pm.y, po.x, po.y, alpha);")
src = src.replace("                mine[pidx(c)] = make_double2(with_sign(m1, hx), with_sign(m2, hz));",
                  "                mine[pidx(c)] = make_double2(with_sign(m1, hx), with_sign(m2, hz));\n                if (shot == 0 && SIDE == 0 && ix == 5) printf(\"part %d hx %x m1 %g w %g\\n\", c, hx, m1, mine[pidx(c)].x);")
src = src.replace("                        c[k] = xor_sign(y * alpha, hi32(v[e]));",
                  "                        c[k] = xor_sign(y * alpha, hi32(v[e]));\n                        if (shot == 0 && SIDE == 0 && ix == 5) printf(\"q %d k %d r %d y %g c %g\\n\", q, k, r, y, c[k]);")
_abi.check(dec._lib.qd_graph_hgp_replace_source(dec._handle, src.encode()), "replace")
sd = torch.from_numpy(syn).cuda()
x = torch.zeros((B, 225), dtype=torch.uint8, device="cuda:0")
it = torch.zeros(B, dtype=torch.int32, device="cuda:0")
st = torch.zeros(B, dtype=torch.uint8, device="cuda:0")
_abi.check(dec._lib.qd_graph_hgp_decode_bp(dec._handle, B, sd.data_ptr(), x.data_ptr(), it.data_ptr(),
                                           st.data_ptr(), 1, 0.0, None), "hgp")
torch.cuda.synchronize()
print("syn ptr", hex(sd.data_ptr()), "x sum", int(x.sum()))
