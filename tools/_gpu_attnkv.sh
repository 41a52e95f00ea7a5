set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attn or attention" > gpurun_out/attnkv_tests.log 2>&1 || { tail -30 gpurun_out/attnkv_tests.log; exit 1; }
tail -3 gpurun_out/attnkv_tests.log
timeout -k 10 120 python -u tools/attn_bwd_time.py > gpurun_out/attnkv_time.log 2>&1 || { cat gpurun_out/attnkv_time.log; exit 1; }
cat gpurun_out/attnkv_time.log
for m in ${MODELS:-}; do
  for a in 1 0; do
    SKP_ATTN_FUSED_KV=$a timeout -k 10 400 python -u bench.py --model $m --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/ab_$m$a.json 2> gpurun_out/ab_$m$a.err || { tail -20 gpurun_out/ab_$m$a.err; exit 1; }
    echo "$m fused=$a $(python -c "import json;d=json.loads(open('gpurun_out/ab_$m$a.json').read().strip().splitlines()[-1]);print(d['value'], d['config'].get('tuned_gemms'))")"
  done
done
