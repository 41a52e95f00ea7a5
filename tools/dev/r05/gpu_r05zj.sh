#!/bin/bash
# r05zj: same-box check of the generalised pair grid (HEAD) against the build before it (b940989)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
KB=mapssel8 RUN_TAG=r05zj ROUNDS=3 bash tools/gpu_kb_env.sh SKP_NONE=1 SKP_LIB=$GRAFT_REPO_ROOT/stablekeypoints_amd/libskp_base.so || exit 1
echo r05zj-ok
