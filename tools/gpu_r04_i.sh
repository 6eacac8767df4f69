#!/bin/bash
# r04 batch i: SE probe (bf16) under a load process running this library in fp32 (no LDS-DMA GEMM kernels)
mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > gpurun_out/r04i_$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
P=$PWD/rcnn-ocr_amd/crnn_hip/libcrnn_hip_seprobe.so
SE_PROBE_LOAD=fp32 CRNN_HIP_LIB=$P step probe_fp32load timeout -k 10 300 python -u tools/se_probe.py 40
SE_PROBE_LOAD=fp32 CRNN_HIP_LIB=$P step probe_fp32load2 timeout -k 10 300 python -u tools/se_probe.py 40
CRNN_HIP_LIB=$P step probe_bf16load timeout -k 10 300 python -u tools/se_probe.py 40
