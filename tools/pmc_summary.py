"""Per-kernel average of every PMC counter in rocprofv3 counter_collection CSVs (dev tool).

usage: python tools/pmc_summary.py DIR [--match capture_maps]
Prints, per kernel name (substring filter), the mean counter value per dispatch and the
derived VALU-busy / LDS figures used in DESIGN.md (SQ_* quad-cycle counters, GRBM summed
over the 8 XCDs; 256 CUs).
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    args = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(args.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if args.match and args.match not in k:
                continue
            name = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:90]
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(k)
        for c in sorted(m):
            print(f"  {c:28s} {m[c]:16.1f}  (n={len(cs[c])})")
        cu = 256
        if "GRBM_GUI_ACTIVE" in m:
            cyc = m["GRBM_GUI_ACTIVE"] / 8          # per-XCD GPU-busy cycles
            if "SQ_ACTIVE_INST_VALU" in m:
                # SQ_ACTIVE_INST_VALU counts quad-cycles per SIMD summed over the chip
                print(f"  VALU busy                    {100 * 4 * m['SQ_ACTIVE_INST_VALU'] / (cu * 4 * cyc):6.1f} %")
            if "SQ_INSTS_VALU" in m:
                print(f"  VALU insts / SIMD-cycle      {m['SQ_INSTS_VALU'] / (cu * 4 * cyc):6.3f}")
            if "SQ_LDS_IDX_ACTIVE" in m:
                print(f"  LDS array busy               {100 * m['SQ_LDS_IDX_ACTIVE'] / (cu * cyc):6.1f} %")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                print(f"  MFMA busy                    {100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (cu * 4 * cyc):6.1f} %")
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
            print(f"  LDS bank-conflict share      {100 * m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:6.1f} %")


if __name__ == "__main__":
    main()
