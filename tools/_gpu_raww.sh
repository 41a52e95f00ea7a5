set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/conv_tests.log 2>&1 || { tail -30 gpurun_out/conv_tests.log; exit 1; }
tail -1 gpurun_out/conv_tests.log
for r in 1 0; do
  SKP_WINO_RAWW=$r timeout -k 10 200 python -u tools/conv8_probe.py > gpurun_out/c8r.log 2>&1 || { tail -20 gpurun_out/c8r.log; exit 1; }
  echo "raww=$r: $(grep 'C=' gpurun_out/c8r.log | cut -c1-60 | tr '\n' ' ')"
done
for a in 1 0 1 0; do
  SKP_WINO_RAWW=$a timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/rw.log 2>&1 || exit 2
  echo "raww=$a: $(tail -1 gpurun_out/rw.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'])")"
done
