# Re-tune the SD15 bench's GEMM shapes with a longer per-solution budget, then A/B against the shipped table.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
date +%s > gpurun_out/t0
SKP_TUNED_GEMMS=0 PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \
PYTORCH_TUNABLEOP_FILENAME=$GRAFT_REPO_ROOT/gpurun_out/retune%d.csv \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-30} PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
timeout -k 10 800 python -u bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/retune.log 2>&1 || { echo tune failed; tail -5 gpurun_out/retune.log; exit 1; }
echo "tuning took $(( $(date +%s) - $(cat gpurun_out/t0) )) s"; wc -l gpurun_out/retune0.csv
for i in 1 2; do
  SKP_TUNED_GEMMS_FILE=$GRAFT_REPO_ROOT/gpurun_out/retune0.csv timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/rt.log 2>&1 || exit 2
  echo "retuned: $(tail -1 gpurun_out/rt.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['config']['tuned_gemms'])")"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/rt.log 2>&1 || exit 3
  echo "shipped: $(tail -1 gpurun_out/rt.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['config']['tuned_gemms'])")"
done
