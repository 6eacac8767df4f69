#!/bin/bash
# r05m: determinism beside this library's own step, DP tests without turn-taking (two processes compute at once)
set -o pipefail
o=gpurun_out/r05m
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_dp.py tests/test_train_dp.py -x -v -s --timeout 300 --timeout-method thread > $o/det_dp_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error|rank [01]:" $o/det_dp_tests.log | tail -n 30
exit $rc
