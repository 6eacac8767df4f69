#!/bin/bash
# r03y: pack / BiLSTM / train-step GPU tests, the train bench and its rocprof summary, then the
# strided-dgrad persistence A/B (per-class launches with CRNN_OPT_GEMM_PERSISTENT off / on)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r03y}
mkdir -p gpurun_out
TAG=$T PYTEST_K="$PYTEST_K" PYTEST_PATHS="$PYTEST_PATHS" bash tools/gpu_r03_quick.sh > gpurun_out/${T}_quick.log 2>&1 || { tail -20 gpurun_out/${T}_quick.log; exit 1; }
grep -E "passed|^bench" gpurun_out/${T}_quick.log; grep pack gpurun_out/${T}_summary.md | cut -c1-110
for l in 2 5; do
  timeout -k 10 120 python -u tools/kbench.py --only dgrad --layer $l --opt 16=1,0 >> gpurun_out/${T}_dgrad_ab.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/kbench.py --only dgrad --layer $l --set 16=0 --opt 1=0,1,0,1 >> gpurun_out/${T}_dgrad_ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/${T}_dgrad_ab.log | grep -v "^sum"
