set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/pd.log 2>&1 || { tail -20 gpurun_out/pd.log; exit 2; }
  echo "edge pad: $(tail -1 gpurun_out/pd.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'])")"
done
