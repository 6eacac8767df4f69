#!/bin/bash
# gemm_square.py over library variants: VARIANTS="lib:opt ..." (lib empty = libcrnn_hip.so)
cd $GRAFT_REPO_ROOT
for v in $VARIANTS; do
  lib=${v%%:*}; opt=${v##*:}
  if [ -n "$lib" ]; then export CRNN_HIP_LIB=$PWD/rcnn-ocr_amd/crnn_hip/$lib; else unset CRNN_HIP_LIB; fi
  timeout -k 10 120 python -u tools/gemm_square.py $opt > gpurun_out/gv.log 2>&1 || { cat gpurun_out/gv.log; exit 1; }
  echo "== $v"; grep " TF " gpurun_out/gv.log
done
