set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "layer_norm" > gpurun_out/ln_tests.log 2>&1 || { tail -30 gpurun_out/ln_tests.log; exit 1; }
tail -1 gpurun_out/ln_tests.log
timeout -k 10 120 python -u - > gpurun_out/ln_time.log 2>&1 <<'PY' || { cat gpurun_out/ln_time.log; exit 1; }
import torch
from stablekeypoints_amd import ops
for shape in ((8, 4096, 320), (8, 1024, 640), (8, 256, 1280)):
    x = torch.randn(*shape, device="cuda:0"); w = torch.randn(shape[-1], device="cuda:0"); b = torch.randn_like(w)
    def t(f, it=50):
        f(); torch.cuda.synchronize()
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(it): f()
        e.record(); torch.cuda.synchronize(); return a.elapsed_time(e) / it * 1e3
    t1 = t(lambda: ops.layer_norm(x, w, b, 1e-5)); t0 = t(lambda: torch.nn.functional.layer_norm(x, (shape[-1],), w, b, 1e-5))
    print(shape, f"skp {t1:.1f} us ({2*x.numel()*4/t1/1e3:.0f} GB/s)  torch {t0:.1f} us")
PY
cat gpurun_out/ln_time.log
for a in 1 0 1 0; do
  SKP_LN=$a timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/ln.log 2>&1 || { tail -20 gpurun_out/ln.log; exit 2; }
  echo "ln=$a: $(tail -1 gpurun_out/ln.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'])")"
done
