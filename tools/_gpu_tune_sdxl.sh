set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export SKP_TUNED_GEMMS=0
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1
export PYTORCH_TUNABLEOP_FILENAME=$GRAFT_REPO_ROOT/gpurun_out/tunableop_sdxl%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=10 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=2
timeout -k 10 1000 python -u bench.py --model sdxl --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/tune_sdxl.log 2>&1 || { tail -5 gpurun_out/tune_sdxl.log; exit 1; }
wc -l gpurun_out/tunableop_sdxl0.csv
