set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $GRAFT_REPO_ROOT/gpurun_out/prof -o r01 --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1; echo "prof rc=$?"
cd $GRAFT_REPO_ROOT; tail -3 gpurun_out/gpu_tests.log; find gpurun_out/prof -name "*stats*"
