set -o pipefail
cd $GRAFT_REPO_ROOT
S="8,320,320,64;8,640,320,64;8,320,640,64;8,640,640,32;8,1280,640,32;8,640,1280,32;8,1280,1280,16;8,2560,1280,16;8,1280,1280,8;8,2560,1280,8"
for n in 1 2 4 5 8 10 16; do echo "nsplit=$n"; SKP_WINO_NSPLIT=$n timeout -k 10 120 python -u tools/wino_time.py --shapes "$S" || exit 9; done
echo auto; timeout -k 10 120 python -u tools/wino_time.py --shapes "$S"
