#!/bin/bash
# PMC A/B of one kbench entry (KB) under environment settings: each counter set (PASSES, ';'-separated
# lists) in its own run under `timeout -s KILL`, per the MI355X guide's rocprofv3 rules:
#   KB=maps8 PASSES="SQ_WAIT_ANY SQ_WAVE_CYCLES;SQ_INSTS_LDS" bash tools/gpu_pmc_ab.sh "SKP_X=0" "SKP_X=1"
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/${RUN_TAG:-pmcab}
mkdir -p $O
cd /tmp
i=0
for e in "$@"; do
  i=$((i+1))
  p=0
  IFS=';' read -ra SETS <<< "$PASSES"
  for cs in "${SETS[@]}"; do
    p=$((p+1))
    export $e
    timeout -s KILL 90 rocprofv3 --pmc $cs --kernel-trace -d $O/v${i}_p$p -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only $KB --iters 3 > $O/v${i}_p$p.log 2>&1 || { echo "pmc ($e / $cs) failed"; tail -5 $O/v${i}_p$p.log; exit 12; }
    unset ${e%%=*}
  done
  echo "== $e"
  python3 $ROOT/tools/pmc_table.py $(find $O -path "*v${i}_p*" -name "*counter_collection.csv") --kernel ${KNAME:-capture_maps}
done
echo pmcab-ok
