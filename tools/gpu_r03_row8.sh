#!/bin/bash
# r03: conv kernel tests on the row8-epilogue build, then A/B vs the build without it (bench + kbench)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or train_step or eval or halo" > gpurun_out/r03e_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03e_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r03e_pytest.log | head; exit 1; }
LIB_B=rcnn-ocr_amd/crnn_hip/libcrnn_hip_norow8.so KB=1 bash tools/gpu_lib_ab.sh > gpurun_out/r03e_ab.log 2>&1
rc=$?; cat gpurun_out/r03e_ab.log; exit $rc
