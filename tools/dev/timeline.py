"""Dev: timeline of one overlapped headline step from a rocprofv3 kernel trace
of bench.py (a rocprofv3 --kernel-trace run of bench.py; its round-3 launcher was removed in round 6).  Prints each BP / SSF kernel's start,
end and queue relative to the step's first start."""
import csv, sys
from collections import defaultdict
trace = sys.argv[1]
step = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows = list(csv.DictReader(open(trace)))
print("columns:", list(rows[0].keys()))
bp = sorted([r for r in rows if "bp_ms_wave_kernel<double" in r["Kernel_Name"] and r["Kernel_Name"].split(">(")[0].endswith(", 3")],
            key=lambda r: int(r["Start_Timestamp"]))
ssf = sorted([r for r in rows if "ssf_wave_kernel" in r["Kernel_Name"]], key=lambda r: int(r["Start_Timestamp"]))
P = 9
sel = bp[step * P:(step + 1) * P] + ssf[step * P:(step + 1) * P]
t0 = min(int(r["Start_Timestamp"]) for r in sel)
t1 = max(int(r["End_Timestamp"]) for r in sel)
q = next((k for k in ("Queue_Id", "Stream_Id", "Queue_ID") if k in rows[0]), None)
for r in sorted(sel, key=lambda r: int(r["Start_Timestamp"])):
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    kind = "BP " if "bp_ms" in r["Kernel_Name"] else "SSF"
    print(f"{kind} q={r.get(q) if q else '?'} start {s/1e6:7.3f} end {e/1e6:7.3f} dur {(e-s)/1e6:6.3f} ms")
print(f"step span {(t1-t0)/1e6:.3f} ms")
# concurrency profile
ev = sorted([(int(r["Start_Timestamp"]), 1) for r in sel] + [(int(r["End_Timestamp"]), -1) for r in sel])
cur, last, hist = 0, t0, defaultdict(float)
for t, d in ev:
    hist[cur] += (t - last) / 1e6
    cur += d
    last = t
print("time at k concurrent kernels (ms):", {k: round(v, 3) for k, v in sorted(hist.items())})
