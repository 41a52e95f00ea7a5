set -o pipefail
cd $GRAFT_REPO_ROOT
for d in 0 4 8 12 5 13; do
  echo "dbg=$d"
  SKP_WINO_DEBUG=$d timeout -k 10 120 python -u tools/wino_time.py --shapes "8,128,128,512;8,512,512,64" || exit 9
done
