"""HBM traffic per launch of a kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Both counters are in KB.  On gfx950 FETCH_SIZE reports half of wide coalesced reads, so it is
doubled (MI355X_MICROARCH.md, HBM/rocprofv3 section); WRITE_SIZE is taken as is.  The median
over launches is used (the first launch also pays cold TLB misses).

usage: python tools/pmc_traffic.py FETCH.csv WRITE.csv --kernel aggregate_kernel \
           --algorithmic 1081344000 --out profiles/pmc_traffic.json
"""
import argparse
import csv
import json
import statistics


def values(path, kernel, counter, launches=None):
    """Counter values of the kernel's launches in dispatch order; ``launches`` = (a, b) keeps the
    a-th … (b−1)-th of them (one kbench case of several that launch the same kernel)."""
    out = []
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            out.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = [v for _, v in sorted(out)]
    if launches:
        out = out[launches[0]:launches[1]]
    if not out:
        raise SystemExit(f"no {counter} rows for {kernel} in {path}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--kernel", default="aggregate_kernel")
    ap.add_argument("--name", default="skp_aggregate")
    ap.add_argument("--algorithmic", type=int, default=1081344000)
    ap.add_argument("--out", default=None, help="JSON file to update (other kernels' entries are kept)")
    ap.add_argument("--workload", default="tools/kbench.py --only agg (N=500, R=128, 4 distinct layers x 8 heads)")
    ap.add_argument("--launches", default="", help="a:b = the kernel's a-th … (b−1)-th launches in dispatch order")
    args = ap.parse_args()
    rng = tuple(int(x) for x in args.launches.split(":")) if args.launches else None
    f = values(args.fetch, args.kernel, "FETCH_SIZE", rng)
    w = values(args.write, args.kernel, "WRITE_SIZE", rng)
    fm, wm = statistics.median(f), statistics.median(w)
    fetch = fm * 1024 * 2
    write = wm * 1024
    res = {args.name: {
        "hbm_bytes_per_launch": fetch + write,
        "fetch_bytes_corrected": fetch,
        "write_bytes": write,
        "fetch_size_kb_raw_median": fm,
        "write_size_kb_raw_median": wm,
        "algorithmic_bytes_per_launch": args.algorithmic,
        "traffic_over_algorithmic": (fetch + write) / args.algorithmic,
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes on "
                  f"{args.workload}; FETCH_SIZE (KB) x1024 x2 "
                  "(gfx950: FETCH_SIZE reports half of wide coalesced reads, MI355X_MICROARCH.md HBM section), "
                  "WRITE_SIZE (KB) x1024; median over launches (tools/pmc_traffic.py)",
        "launches": min(len(f), len(w)),
    }}
    print(json.dumps(res, indent=1))
    if args.out:
        try:
            allrec = json.load(open(args.out))
        except (OSError, ValueError):
            allrec = {}
        allrec.update(res)
        open(args.out, "w").write(json.dumps(allrec, indent=1) + "\n")


if __name__ == "__main__":
    main()
