#!/bin/bash
# r04 batch g: SE probe under a bench.py load, this process's allocations shifted (SE_PROBE_SHIFT=1) vs not
mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > gpurun_out/r04g_$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
P=$PWD/rcnn-ocr_amd/crnn_hip/libcrnn_hip_seprobe.so
SE_PROBE_SHIFT=1 CRNN_HIP_LIB=$P step probe_shift timeout -k 10 300 python -u tools/se_probe.py 40
CRNN_HIP_LIB=$P step probe_noshift timeout -k 10 300 python -u tools/se_probe.py 40
SE_PROBE_SHIFT=1 CRNN_HIP_LIB=$P step probe_shift2 timeout -k 10 300 python -u tools/se_probe.py 40
