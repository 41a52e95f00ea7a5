"""Gaps on the main stream of a bench timed region (rocprofv3 kernel trace): how long the main stream
sits idle between kernels, by size, and the largest gaps with their neighbours (dev tool).

    python tools/stream_gaps.py TRACE.csv [--steps 2]
"""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--top", type=int, default=15)
args = ap.parse_args()
rows = list(csv.DictReader(open(args.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "multi_tensor_apply" in r["Kernel_Name"]]
groups = []
for i in adam:
    if groups and i - groups[-1][-1] <= 16:
        groups[-1].append(i)
    else:
        groups.append([i])
sel = rows[groups[-args.steps - 1][-1] + 1:]
main = [r for r in sel if r["Stream_Id"] == "0"]
gaps = []
for a, b in zip(main, main[1:]):
    g = int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
    gaps.append((g, a["Kernel_Name"][:48], b["Kernel_Name"][:48]))
hist = collections.Counter()
for g, _, _ in gaps:
    if g > 0:
        hist["<5us" if g < 5000 else "<20us" if g < 20000 else "<100us" if g < 100000 else "<1ms" if g < 1e6 else ">1ms"] += g
print(f"main-stream gaps: {sum(g for g, _, _ in gaps if g > 0) / 1e6:.2f} ms over {args.steps} steps; by size (ms):",
      {k: round(v / 1e6, 2) for k, v in sorted(hist.items())})
for g, a, b in sorted(gaps, reverse=True)[:args.top]:
    print(f"{g / 1e3:9.1f} us  after {a:48s} before {b}")
