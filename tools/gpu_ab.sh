#!/bin/bash
# A/B runs of bench.py variants; each run under its own limit, stops at the first failure.
# usage: bash tools/gpu_ab.sh "<args A>" "<args B>" ...
set -o pipefail
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $a > gpurun_out/ab_$i.log 2>&1 || { echo "run $i ($a) failed rc=$?"; tail -20 gpurun_out/ab_$i.log; exit 1; }
  echo "[$a] $(tail -1 gpurun_out/ab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],2), "img/s", round(d["ms_per_step"],1), "ms/step")')"
done
