#!/bin/bash
# r04: upper bound of a halo-staged A operand for the 3x3 convs: kbench fwd with the A LDS-DMA issued
# for the first 8 K-tiles only (diagnostic build, results invalid) vs the default library
mkdir -p gpurun_out
for rep in 1 2; do
  for L in libcrnn_hip.so libcrnn_hip_diagA.so; do
    echo "== $L rep $rep"
    CRNN_HIP_LIB=$PWD/rcnn-ocr_amd/crnn_hip/$L timeout -k 10 120 python -u tools/kbench.py --iters 20 --only fwd 2>&1 | grep -v amdgpu || exit 1
  done
done
