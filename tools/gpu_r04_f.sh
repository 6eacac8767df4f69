#!/bin/bash
# r04 batch f: the DP tests (ranks in turns, exact bar) and the SE probe under a bench.py load and under
# a pure torch.matmul load
mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > gpurun_out/r04f_$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step dp timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_dp.py
P=$PWD/rcnn-ocr_amd/crnn_hip/libcrnn_hip_seprobe.so
CRNN_HIP_LIB=$P step probe_bench timeout -k 10 300 python -u tools/se_probe.py 40
SE_PROBE_LOAD=matmul CRNN_HIP_LIB=$P step probe_matmul timeout -k 10 300 python -u tools/se_probe.py 40
