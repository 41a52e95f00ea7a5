set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attn or attention" > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/rg.log 2>&1 || exit 2
  echo "ragged flash: $(tail -1 gpurun_out/rg.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'])")"
done
