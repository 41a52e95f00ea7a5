#!/bin/bash
# re-tune the GEMM table on the current tree (new head-major cross-attention shapes), then bench
# A/B: the re-tuned table vs the shipped one (alternating)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/${RUN_TAG:-r03au}
mkdir -p $O
cd $ROOT
bash tools/tune_gemms.sh || { echo "tuning failed"; exit 1; }
cp gpurun_out/tunableop_results0.csv $O/gemm_retuned.csv
grep -c "" $O/gemm_retuned.csv
for i in 1 2; do
  for t in new old; do
    F=""; [ $t = new ] && F=$O/gemm_retuned.csv
    timeout -k 10 400 env SKP_TUNED_GEMMS_FILE=$F python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_${t}_$i.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_${t}_$i.log; exit 4; }
    tail -1 $O/bench_${t}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', round(d['value'],3), round(d['ms_per_step'],2), d['config']['tuned_gemms'])"
  done
done
