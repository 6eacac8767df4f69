#!/bin/bash
# r03: kernel tests for the forward-path dgrad, then per-layer conv A/B: native dgrad vs forward-path
# dgrad, and the epilogue-store cost (CRNN_OPT_DIAG bit 0) of fwd / dgrad / wgrad
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r03kb}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -rP --timeout 120 --timeout-method thread -k "tw_forward_path or dgrad_bnrelu or conv_" > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/${T}_pytest.log | head; exit 1; }
timeout -k 10 300 python -u tools/kbench.py --only dgrad,dgradtw > gpurun_out/${T}_tw.log 2>&1 || { tail gpurun_out/${T}_tw.log; exit 1; }
cat gpurun_out/${T}_tw.log
timeout -k 10 300 python -u tools/kbench.py --opt 15=0,1 > gpurun_out/${T}_nostore.log 2>&1 || { tail gpurun_out/${T}_nostore.log; exit 1; }
cat gpurun_out/${T}_nostore.log
