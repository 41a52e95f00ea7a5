#!/bin/bash
# r05zf: paired sel_dense grid of 16-wave blocks (s = 32 jobs on whole-wave bands, two s = 16 jobs
# per block) vs the 8-wave paired grid (half-wave bands at R/s = 4, build SKP_SEL_LW4=32) (dev)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05zf; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sel_bwd.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u - > $O/equal.log 2>&1 <<'PY' || { echo "equality check failed"; tail -5 $O/equal.log; exit 1; }
# the new grid against the old one, same inputs (subprocess with SKP_LIB per build): bit equality
import os, subprocess, sys
code = r'''
import sys, torch, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden")
import test_gpu_sel_bwd as t
zs, tok, gsel = t._case(5, 8, 8, (16, 16, 16, 32), 128, 500, 10)
zt = [t.T(z) for z in zs]
_, stats = t._fwd(zt, [16, 16, 16, 32], 8, 8, 128)
out = t._sel_abi(zt, [16, 16, 16, 32], 8, 8, 128, t.T(tok), t.T(gsel), 0.03125, stats)
np.savez(sys.argv[1], *[o.cpu().numpy() for o in out])
'''
env = dict(os.environ)
subprocess.run([sys.executable, "-c", code, "/tmp/new.npz"], check=True, env=env)
env["SKP_LIB"] = os.path.join(os.environ["GRAFT_REPO_ROOT"], "build/var_lw32/libskp.so")
subprocess.run([sys.executable, "-c", code, "/tmp/old.npz"], check=True, env=env)
import numpy as np
a, b = np.load("/tmp/new.npz"), np.load("/tmp/old.npz")
same = all(np.array_equal(a[k], b[k]) for k in a.files)
print("bit-identical to the 8-wave grid:", same, [float(np.abs(a[k] - b[k]).max()) for k in a.files])
PY
cat $O/equal.log | tail -1
KB=mapssel8 RUN_TAG=r05zf ROUNDS=3 bash tools/gpu_kb_env.sh SKP_NONE=1 SKP_LIB=$GRAFT_REPO_ROOT/build/var_lw32/libskp.so || exit 1
KB=mapssel8 RUN_TAG=r05zf_prof bash tools/gpu_kb_prof_env.sh SKP_NONE=1 || exit 1
echo r05zf-ok
