#!/bin/bash
# r05t: word accuracy on the generalising reference model (10 000 held-out lines) + DP run_training with BN statistics
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_refmodel.py tests/test_train_dp.py > gpurun_out/r05t_refmodel.log 2>&1
rc=$?
grep -E "held-out|fit |val |DP vs|BN running|passed|failed|FAILED|Error" gpurun_out/r05t_refmodel.log | head -40
exit $rc
