set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/conv8_probe.py > gpurun_out/conv8.log 2>&1 || { tail -20 gpurun_out/conv8.log; exit 1; }
TUNE=1 timeout -k 10 300 python -u tools/conv8_probe.py > gpurun_out/conv8_tuned.log 2>&1 || { tail -20 gpurun_out/conv8_tuned.log; exit 1; }
grep "C=" gpurun_out/conv8.log; echo tuned:; grep "C=" gpurun_out/conv8_tuned.log
