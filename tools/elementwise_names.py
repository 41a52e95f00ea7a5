"""Group the strided / elementwise / transpose kernels of a rocprofv3 kernel trace (run WITHOUT -T, so
the names carry their functor types) by (name, grid), largest total first (dev tool)."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r["Kernel_Name"]
    if "elementwise" in n or "transpose" in n or "copy" in n.lower() or "reduce" in n:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        key = (re.sub(r"\s+", " ", n)[:900], r["Grid_Size_X"], r["Stream_Id"])
        agg[key][0] += 1
        agg[key][1] += d
for (n, g, s), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:80]:
    print(f"{t / 1e3:8.3f} ms {c:4d} grid {g:>10s} stream {s}  {n}")
