#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03aa
mkdir -p $O
cd $ROOT
run() { timeout -k 10 120 env "$@" python -u tools/miopen_s2_probe.py >> $O/probe.log 2>&1 || { echo "probe failed: $*"; tail -5 $O/probe.log; exit 1; }; }
run PROBE_TAG=default
timeout -k 10 300 env PROBE_TAG=default python -u tools/miopen_s2_probe.py --find >> $O/probe.log 2>&1 || { echo "find failed"; exit 2; }
run PROBE_TAG=no_nhwc_gtc MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0
run PROBE_TAG=no_igemm MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=0
run PROBE_TAG=no_igemm_no_gemm MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=0 MIOPEN_DEBUG_CONV_GEMM=0
run PROBE_TAG=no_igemm_no_direct MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=0 MIOPEN_DEBUG_CONV_DIRECT=0
grep -v amdgpu $O/probe.log
