set -o pipefail
cd $GRAFT_REPO_ROOT
for o in 1 2; do echo "order=$o"; SKP_WINO2_ORDER=$o timeout -k 10 120 python -u tools/wino_time.py --shapes "8,128,128,512;8,128,256,256;8,256,256,256;8,512,512,128;8,512,512,64" || exit 9; done
