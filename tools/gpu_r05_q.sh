#!/bin/bash
# r05q: BiLSTM / linear GEMM entry points vs hipBLASLt at the bench shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
GEMMBENCH_VENDOR=1 timeout -k 10 200 python -u tools/gemmbench.py 2=0,1 > gpurun_out/r05q_gemmbench.log 2>&1; rc=$?
cat gpurun_out/r05q_gemmbench.log; exit $rc
