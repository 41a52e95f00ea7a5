set -o pipefail
cd $GRAFT_REPO_ROOT
S="8,128,128,512;8,256,256,256;8,512,512,128;8,512,512,64;8,320,320,64;8,640,640,32"
for d in 16 32 48 15 47; do echo "dbg=$d"; SKP_WINO2_DEBUG=$d timeout -k 10 120 python -u tools/wino_time.py --shapes "8,128,128,512;8,512,512,64" || exit 9; done
for o in 1 2; do echo "order=$o"; SKP_WINO2_ORDER=$o timeout -k 10 120 python -u tools/wino_time.py --shapes "$S" || exit 9; done
