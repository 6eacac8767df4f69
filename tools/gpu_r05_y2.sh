#!/bin/bash
# r05y2: per-layer A/B of the remaining tuning switches (GEMM stagger, W-halo, pad skip) over every conv geometry
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for o in "0=1,0,1,0" "18=1,0,1,0" "11=1,0,1,0"; do
  timeout -k 10 240 python -u tools/kbench.py --iters 10 --opt $o > gpurun_out/r05y2_kbench_opt${o%%=*}.log 2>&1 || { tail -5 gpurun_out/r05y2_kbench_opt${o%%=*}.log; exit 1; }
  echo "== opt $o"; grep -v amdgpu.ids gpurun_out/r05y2_kbench_opt${o%%=*}.log | tail -12
done
