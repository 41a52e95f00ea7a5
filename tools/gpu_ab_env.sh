#!/bin/bash
# A/B of bench.py under environment settings, alternating, each run under its own limit:
#   bash tools/gpu_ab_env.sh "SKP_X=0" "SKP_X=1" [...]   (ROUNDS alternations, default 2; ARGS: bench args)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${RUN_TAG:-ab}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline ${ARGS:-} > $O/ab_${r}_$i.log 2>&1 || { echo "run ($e) failed rc=$?"; tail -20 $O/ab_${r}_$i.log; exit 1; }
    echo "[$e] $(grep '{"metric"' $O/ab_${r}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],2), "img/s", round(d["ms_per_step"],1), "ms/step")')"
  done
done
