#!/bin/bash
# A/B of kbench entries (KB, comma list) under environment settings, alternating ROUNDS times
# (default 2), each run under its own limit; stops at the first failure:
#   KB=maps8 bash tools/gpu_kb_env.sh "SKP_X=0" "SKP_X=1" [...]
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${RUN_TAG:-kbab}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 python -u tools/kbench.py --only $KB --iters ${KB_ITERS:-20} > $O/kb_${r}_$i.log 2>&1 || { echo "run ($e) failed rc=$?"; tail -20 $O/kb_${r}_$i.log; exit 1; }
    echo "[$e] $(grep -v amdgpu $O/kb_${r}_$i.log | tail -3 | tr '\n' ' ')"
  done
done
