#!/bin/bash
# A/B of the BSHD attention: micro timings, then timed-region kernel summaries of the bench with and
# without it (same box).
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03d
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u tools/attn_bshd_time.py > $O/attn.log 2>&1 || { echo "attn failed"; tail -20 $O/attn.log; exit 1; }
cat $O/attn.log | grep -v amdgpu.ids
cd /tmp
for v in 1 0; do
  SKP_ATTN_BSHD=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof$v -o bench --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/prof$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/prof$v.log; exit 2; }
  cd $ROOT && python3 tools/prof_summary.py $O/prof$v/bench_kernel_trace.csv --steps 2 --accum 4 --out $O/timed$v.csv --top 30 > $O/timed$v.txt || { echo "summary failed"; exit 3; }
  head -14 $O/timed$v.txt
  cd /tmp
done
echo all-ok
