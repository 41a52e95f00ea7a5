"""VALU-busy of one kernel from a rocprofv3 PMC pass (SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE), merged
into a JSON record keyed by kernel (dev tool; bench.py reports it beside the VALU roofline).

VALU busy = 4·SQ_ACTIVE_INST_VALU (quad-cycles, summed over the chip) / (1024 SIMDs · GRBM_GUI_ACTIVE/8)
(GRBM_GUI_ACTIVE is summed over the 8 XCDs); median over launches.

usage: python tools/pmc_valu.py COUNTERS.csv --kernel capture_maps_kernel --name skp_capture_maps_fwd \
           --flop 34078720000 --out profiles/pmc_valu.json

``--kernel a,b,c``: one call made of several kernels (skp_capture_maps_bwd_sel = sel_gather, sel_dot,
sel_adj, sel_dense): the call's VALU-busy is Σ 4·ACTIVE_INST_VALU / Σ 1024·GRBM_GUI_ACTIVE/8 over
its kernels (each kernel's median launch), i.e. weighted by their active time.
"""
import argparse
import csv
import collections
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--name", required=True)
    ap.add_argument("--flop", type=int, required=True, help="algorithmic FLOP per launch (ops.capture_maps_flops)")
    ap.add_argument("--workload", default="")
    ap.add_argument("--out", default=None)
    ap.add_argument("--launches", default="", help="a:b = each kernel's a-th … (b−1)-th launches in dispatch order")
    args = ap.parse_args()
    sel = tuple(int(v) for v in args.launches.split(":")) if args.launches else None
    names = [k for k in args.kernel.split(",") if k]
    per = {k: collections.defaultdict(dict) for k in names}
    for r in csv.DictReader(open(args.csv)):
        for k in names:
            if k in r["Kernel_Name"]:
                per[k][r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    def launch_rows(k):
        rows = [per[k][i] for i in sorted(per[k], key=int)
                if "SQ_ACTIVE_INST_VALU" in per[k][i] and per[k][i].get("GRBM_GUI_ACTIVE")]
        return rows[sel[0]:sel[1]] if sel else rows

    num = den = 0.0
    counts = []
    for k in names:
        rows = launch_rows(k)
        if not rows:
            raise SystemExit(f"no counters for {k}")
        counts.append(len(rows))
        num += statistics.median(4 * d["SQ_ACTIVE_INST_VALU"] for d in rows)
        den += statistics.median(1024 * d["GRBM_GUI_ACTIVE"] / 8 for d in rows)
    busy = [num / den]
    if len(names) == 1:
        rows = launch_rows(names[0])
        busy = [4 * d["SQ_ACTIVE_INST_VALU"] / (1024 * d["GRBM_GUI_ACTIVE"] / 8) for d in rows]
    rec = {args.name: {"valu_busy": statistics.median(busy), "launches": min(counts), "kernels": names,
                       "flop_per_launch": args.flop,
                       "method": "rocprofv3 --pmc SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE; 4*ACTIVE_INST_VALU / "
                                 "(1024 SIMDs * GRBM_GUI_ACTIVE/8), median over launches; several kernels: active-time weighted (tools/pmc_valu.py)",
                       "workload": args.workload}}
    print(json.dumps(rec, indent=1))
    if args.out:
        try:
            allrec = json.load(open(args.out))
        except (OSError, ValueError):
            allrec = {}
        allrec.update(rec)
        open(args.out, "w").write(json.dumps(allrec, indent=1) + "\n")


if __name__ == "__main__":
    main()
