import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import numpy as np
from conftest import load_checks
from oracle import load as load_oracle
from exp_ldpc_amd.decoder import Decoder
HX, HZ = load_checks("hgp_12_3_4_s1234")
orc = load_oracle()
rng = np.random.default_rng(4)
e = (rng.random((64, 225)) < 0.03).astype(np.uint8)
syn = ((HZ @ e.T).T % 2).astype(np.uint8)
for prec in ("f32", "f64"):
    for mi in (1, 2, 5, 30):
        dec = Decoder(HZ, 0.02, method="ms", precision=prec, max_iter=mi)
        got = dec.decode(syn, want=("x", "llr", "iters", "status"))
        ref = orc.decode(HZ, 0.02, syn, method="ms", precision=prec, max_iter=mi)
        bad = np.nonzero((got["llr"].astype(np.float64) != ref["llr"]).any(1))[0]
        print(prec, mi, "llr-mismatch shots", len(bad), "x-mismatch", int((got["x"] != ref["x"]).any(1).sum()),
              "iters-mismatch", int((got["iters"] != ref["iters"]).sum()))
        if len(bad):
            b = bad[0]
            d = np.nonzero(got["llr"][b].astype(np.float64) != ref["llr"][b])[0]
            print("  shot", b, "cols", d[:10], "got", got["llr"][b][d[:5]], "ref", ref["llr"][b][d[:5]])
