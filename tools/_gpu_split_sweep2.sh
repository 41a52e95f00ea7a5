#!/bin/bash
# Winograd split-K sweep at the UNet's 64²/32²/16² shapes (batch 8) on the current kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
S="8,320,320,64;8,640,320,64;8,960,320,64;8,640,640,32;8,1280,640,32;8,1920,640,32;8,1280,1280,16;8,2560,1280,16"
for n in 2 3 4 5 8 10 16; do echo "nsplit=$n"; SKP_WINO_NSPLIT=$n timeout -k 10 120 python -u tools/wino_time.py --iters 5 --shapes "$S" || exit 9; done
echo auto; timeout -k 10 120 python -u tools/wino_time.py --iters 5 --shapes "$S"
