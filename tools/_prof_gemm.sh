#!/bin/bash
# Kernel-trace durations of the bgemm micro-benchmark (host overhead excluded)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/prof_gemm
mkdir -p $OUT
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT -o g --output-format csv -- python3 $ROOT/tools/kbench.py --only gemm16,gemm32 --iters 20 > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 1; }
cd $ROOT && python3 - <<'PY'
import csv, glob, collections, os
f = glob.glob(os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out/prof_gemm/**/*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(f)))
seq = [(r["Kernel_Name"].split("(")[0].replace("void ", "")[-60:], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
seq = [x for x in seq if "bgemm" in x[0] or "Cijk" in x[0]]
# kbench order: gemm16 (fwd, dq, dk, torch) × 21 calls each, then gemm32
names = ["16_fwd", "16_dq", "16_dk", "16_torch", "32_fwd", "32_dq", "32_dk", "32_torch"]
i = 0
for n in names:
    chunk = seq[i:i + 21]; i += 21
    d = sorted(t for _, t in chunk)[1:-1]
    print(f"{n:9s} {sum(d)/len(d):8.1f} us  ({chunk[0][0][:50]})")
PY
