set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/conv_tests.log 2>&1 || { tail -30 gpurun_out/conv_tests.log; exit 1; }
tail -1 gpurun_out/conv_tests.log
timeout -k 10 200 python -u tools/conv8_probe.py > gpurun_out/conv8w.log 2>&1 || { tail -20 gpurun_out/conv8w.log; exit 1; }
grep "C=" gpurun_out/conv8w.log | cut -c1-120
for a in 1 0 1 0; do
  SKP_WINO_WIDE=$a timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/wd.log 2>&1 || exit 2
  echo "wide=$a: $(tail -1 gpurun_out/wd.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'])")"
done
