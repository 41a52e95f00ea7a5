# A/B of an environment switch on bench.py, alternating runs; usage: VAR=name bash tools/_gpu_ab_env.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do for v in 1 0; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 4 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "$VAR=$v $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],2))')"
done; done
