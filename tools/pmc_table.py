"""Median per-launch value of every PMC counter for the kernels matching a name (dev tool).

usage: python tools/pmc_table.py COUNTERS.csv [COUNTERS2.csv ...] --kernel capture_maps
"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--kernel", required=True)
    args = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in args.csv:
        per = collections.defaultdict(dict)
        names = {}
        for r in csv.DictReader(open(f)):
            if args.kernel in r["Kernel_Name"]:
                per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0][-60:]
        for d, cs in per.items():
            for c, v in cs.items():
                vals[names[d]][c].append(v)
    for k, cs in vals.items():
        print(k)
        for c in sorted(cs):
            print(f"  {c:28s} {statistics.median(cs[c]):16.4g}  (n={len(cs[c])})")


if __name__ == "__main__":
    main()
