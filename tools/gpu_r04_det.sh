#!/bin/bash
# r04: finalize / colsum determinism under load + the ticket A/B. A test failure (rc 1) lets the
# next step run; any other status (fault, abort, time limit) ends the script.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_determinism.py \
  > gpurun_out/r04a_det_tests.log 2>&1
rc=$?; echo "determinism tests rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/det_ab.py 256 > gpurun_out/r04a_det_ab.log 2>&1
rc=$?; echo "det_ab rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "finalize or colsum or se_ or bn_ or ctc" > gpurun_out/r04a_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; exit $rc
