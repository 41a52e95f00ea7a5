"""Per-kernel summary of the TIMED region of a bench run from a rocprofv3 kernel trace.

rocprofv3 --stats counts every dispatch, including the warm-up step in which MIOpen's Find
benchmarks candidate convolution kernels (naive reference kernels among them), so the stats
CSV over-states conv time.  This tool sorts dispatches by start time, splits them into
token-opt micro-iterations at the one-per-micro-step `sort_topk_kernel`, keeps the last
`--micro` micro-iterations (the timed steps × accum) and prints/writes per-kernel totals.

usage: python tools/prof_summary.py TRACE.csv --micro 8 [--out summary.csv]
       python tools/prof_summary.py TRACE.csv --steps 2 --accum 4   # split at the Adam kernels
       python tools/prof_summary.py TRACE.csv --tail-ms 250 --images 24   # the last 250 ms of dispatches
       (the --stage benches: their timed region is the end of the run; --images per region)
(with batched micro-steps the per-image marker no longer bounds the timed region; the
optimiser step's multi_tensor_apply kernels do)
"""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--micro", type=int, default=0, help="micro-iterations in the timed region")
    ap.add_argument("--steps", type=int, default=0, help="optimiser steps in the timed region (Adam marker)")
    ap.add_argument("--accum", type=int, default=4, help="images per optimiser step (with --steps)")
    ap.add_argument("--marker", default="sort_topk_kernel")
    ap.add_argument("--tail-ms", type=float, default=0.0, help="keep the dispatches of the trace's last TAIL_MS")
    ap.add_argument("--images", type=int, default=0, help="images in the --tail-ms region (per-image figure)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--top", type=int, default=30)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if args.tail_ms:
        t_end = max(int(r["End_Timestamp"]) for r in rows)
        start = next(i for i, r in enumerate(rows) if int(r["Start_Timestamp"]) >= t_end - args.tail_ms * 1e6)
        args.micro = args.images or 1
    elif args.steps:
        adam = [i for i, r in enumerate(rows) if "multi_tensor_apply" in r["Kernel_Name"]]
        groups = []   # consecutive Adam kernels of one optimiser step
        for i in adam:
            if groups and i - groups[-1][-1] <= 16:
                groups[-1].append(i)
            else:
                groups.append([i])
        if len(groups) < args.steps + 1:
            raise SystemExit(f"only {len(groups)} optimiser steps for {args.steps}")
        start = groups[-args.steps - 1][-1] + 1
        args.micro = args.steps * args.accum
    else:
        marks = [i for i, r in enumerate(rows) if args.marker in r["Kernel_Name"]]
        if len(marks) < args.micro + 1:
            raise SystemExit(f"only {len(marks)} markers for {args.micro} micro-iterations")
        # the timed region starts right after the marker that ends the last warm-up micro-iteration
        start = marks[-args.micro - 1] + 1
    sel = rows[start:]
    t0 = int(sel[0]["Start_Timestamp"])
    t1 = int(sel[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    for r in sel:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[r["Kernel_Name"]][0] += 1
        agg[r["Kernel_Name"]][1] += d
    total = sum(v[1] for v in agg.values())
    # per stream: kernel busy time and the union of its kernels' intervals (the critical path is
    # the main stream; the VAE prefetch runs on a side stream)
    by_stream = collections.defaultdict(list)
    for r in sel:
        by_stream[r.get("Stream_Id", "0")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for sid, iv in sorted(by_stream.items()):
        iv.sort()
        union, cur = 0, None
        for a, b in iv:
            if cur is None or a > cur[1]:
                if cur:
                    union += cur[1] - cur[0]
                cur = [a, b]
            else:
                cur[1] = max(cur[1], b)
        union += cur[1] - cur[0]
        busy = sum(b - a for a, b in iv)
        print(f"stream {sid}: {len(iv)} dispatches, kernel busy {busy / 1e6:.1f} ms, covered {union / 1e6:.1f} ms")
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    print(f"timed region: {len(sel)} dispatches, span {(t1 - t0) / 1e6:.1f} ms, kernel busy {total / 1e6:.1f} ms, "
          f"{args.micro} micro-iterations -> {total / 1e6 / args.micro:.2f} ms kernel time per image")
    for name, (n, d) in items[: args.top]:
        print(f"{d / 1e6:9.2f} ms {100 * d / total:5.1f}% n={n:6d} avg={d / n / 1e3:9.1f} us  {name[:100]}")
    if args.out:
        with open(args.out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for name, (n, d) in items:
                w.writerow([name, n, d, d / n, 100 * d / total])


if __name__ == "__main__":
    main()
