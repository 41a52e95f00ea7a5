set -o pipefail
cd $GRAFT_REPO_ROOT
for d in ${DBGS:-0 12 13 14 15 47}; do echo "dbg=$d"; SKP_WINO2_DEBUG=$d timeout -k 10 120 python -u tools/wino_time.py --shapes "8,128,128,512;8,512,512,64" || exit 9; done
