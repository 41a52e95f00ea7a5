set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in ${MODELS:-sd15}; do
  for a in ${VALS:-40 0 40 0}; do
    SKP_ATTN_FLASH=$a timeout -k 10 400 python -u bench.py --model $m --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/abf_$m$a.json 2> gpurun_out/abf_$m$a.err || { tail -20 gpurun_out/abf_$m$a.err; exit 1; }
    echo "$m flash=$a $(python -c "import json;d=json.loads(open('gpurun_out/abf_$m$a.json').read().strip().splitlines()[-1]);print(d['value'])")"
  done
done
