"""Instruction mix of the BP iteration loop of one kernel in a hipcc -S dump.

Usage: python tools/dev/isa_loop.py <file.s> <mangled-name-substring> [--print]
Finds the innermost backward branch whose body contains v_med3 (the check
pass) and counts its instructions by class.
"""
import re
import sys
from collections import Counter

src, pat = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(pat) + r"\S*:", l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.size") or re.match(r"^\.Lfunc_end", lines[i]))
body = lines[start:end]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
best = None
for i, l in enumerate(body):
    m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        a = labels[m.group(2)]
        seg = body[a:i + 1]
        if any(("v_med3" in s or "v_min_f64" in s) for s in seg) and (best is None or i - a < best[1] - best[0]):
            best = (a, i)
a, b = best
ins = [l.strip() for l in body[a:b + 1] if l.startswith("\t") and not l.strip().startswith((";", "."))]
ops = [s.split()[0] for s in ins]
cls = Counter()
for o in ops:
    if o.startswith("v_"):
        cls["VALU"] += 1
    elif o.startswith("ds_"):
        cls["LDS"] += 1
    elif o == "s_nop":
        cls["s_nop"] += 1
    elif o.startswith("s_"):
        cls["SALU/branch"] += 1
    elif o.startswith(("global_", "buffer_", "flat_", "scratch_")):
        cls["VMEM"] += 1
print(dict(cls), "total", len(ops))
print(Counter(o for o in ops if o.startswith("v_")).most_common(40))
if "--print" in sys.argv:
    print("\n".join(body[a:b + 1]))
