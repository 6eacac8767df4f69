#!/bin/bash
# conv parity tests, then same-box bench A/B of libcrnn_hip.so vs $LIB_B (alternating)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "conv" > gpurun_out/ct.log 2>&1; rc=$?; tail -3 gpurun_out/ct.log; [ $rc = 0 ] || exit 1
LIB_B=${LIB_B:?} bash tools/gpu_lib_ab.sh
