set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/sp.log 2>&1 || { tail -20 gpurun_out/sp.log; exit 2; }
  echo "default bench run $i: $(tail -1 gpurun_out/sp.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['value'],2), round(d['roofline']['frac'],3))")"
done
