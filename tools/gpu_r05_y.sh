#!/bin/bash
# r05y: per-layer A/B sweep of existing tuning switches over every conv geometry (kbench)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for o in "10=1,0" "1=0,1" "3=0,1,4" "14=0,1" "16=1,0"; do
  timeout -k 10 240 python -u tools/kbench.py --iters 10 --opt $o > gpurun_out/r05y_kbench_opt${o%%=*}.log 2>&1 || { tail -5 gpurun_out/r05y_kbench_opt${o%%=*}.log; exit 1; }
  echo "== opt $o"; grep -v amdgpu.ids gpurun_out/r05y_kbench_opt${o%%=*}.log
done
