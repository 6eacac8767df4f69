#!/bin/bash
# r05 soak: co-scheduled determinism of the final tree's defaults, 2 x 1000 overlapped iterations
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/det_opt.py 15 0,0 1000 > gpurun_out/r05_soak_det.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05_soak_det.log | tail -4; exit $rc
