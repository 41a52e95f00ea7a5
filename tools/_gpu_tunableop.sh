# GEMM TunableOp: tune the bench's GEMM shapes once (results CSV), then bench with the CSV only.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTORCH_TUNABLEOP_ENABLED=1
export PYTORCH_TUNABLEOP_FILENAME=$GRAFT_REPO_ROOT/gpurun_out/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-10}
export PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=2
date +%s > gpurun_out/t0
PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 900 python -u bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/tune.log 2>&1 || { echo tune failed; tail -5 gpurun_out/tune.log; exit 1; }
echo "tuning took $(( $(date +%s) - $(cat gpurun_out/t0) )) s"; ls -la gpurun_out/tunableop_results*.csv; wc -l gpurun_out/tunableop_results*.csv
for i in 1 2; do
  PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 4 > gpurun_out/tb.log 2>&1 || exit 2
  echo "tuned: $(tail -1 gpurun_out/tb.log | cut -c1-120)"
  PYTORCH_TUNABLEOP_ENABLED=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 4 > gpurun_out/tb.log 2>&1 || exit 3
  echo "default: $(tail -1 gpurun_out/tb.log | cut -c1-120)"
done
