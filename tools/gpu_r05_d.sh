#!/bin/bash
# r05d: co-scheduled determinism under the 4-wave GEMM switch (CRNN_OPT_GEMM4W 0 = 8-wave, 2 = the wgrads on 4 waves)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/det_opt.py 14 0,2,0,2 300 > gpurun_out/r05d3_det_gemm4w.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05d3_det_gemm4w.log | tail -8; exit $rc
