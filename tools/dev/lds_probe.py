"""Dev: staged probe of bp_ms_lds_kernel (B shots, max_iter, ssf on/off, graph)."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np
from conftest import load_checks
from exp_ldpc_amd.decoder import Decoder
B, mi, ssf, graph = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3] == "1", sys.argv[4]
if graph == "c4":
    hx, hz = load_checks("hgp_80_3_4_s2025")
else:
    from exp_ldpc_amd.codes import make_check_matrix
    rng = np.random.default_rng(3)
    m, n = 600, 700
    rows, colcount = [], np.zeros(n, int)
    for i in range(m):
        cand = [j for j in rng.permutation(n) if colcount[j] < 4][:int(rng.integers(1, 9))]
        for j in cand:
            colcount[j] += 1
        rows.append(sorted(cand))
    hz, hx = make_check_matrix(rows, n), None
rng = np.random.default_rng(1)
e = (rng.random((B, hz.shape[1])) < 0.02).astype(np.uint8)
syn = ((hz @ e.T).T % 2).astype(np.uint8)
dec = Decoder(hz, 0.02, method="ms", precision="f32", max_iter=mi, flip_sets=hx if ssf else None)
t = time.time()
got = dec.decode(syn, want=("x", "iters", "status"))
print(f"{graph} B={B} max_iter={mi} ssf={ssf} {time.time() - t:.3f}s iters={got['iters'][:8]} status={got['status'][:8]}", flush=True)
if os.environ.get("CHECK"):
    from oracle import load
    ref = load().decode(hz, 0.02, syn, method="ms", precision="f32", max_iter=mi)
    for k in ("x", "iters", "status"):
        print(k, np.array_equal(got[k], ref[k]), flush=True)
