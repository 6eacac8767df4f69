#!/bin/bash
# Same-box A/B of two builds of the library (CRNN_HIP_LIB), alternating: kbench + bench.
#   LIB_B=rcnn-ocr_amd/crnn_hip/libcrnn_hip_r02a.so bash tools/gpu_lib_ab.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
A=rcnn-ocr_amd/crnn_hip/libcrnn_hip.so
B=${LIB_B:?}
for rep in 1 2; do
  for L in $A $B; do
    CRNN_HIP_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/lab.json 2> gpurun_out/lab.err || { echo "bench failed ($L)"; tail -20 gpurun_out/lab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/lab.json')); k=d['kernels']; print('[$(basename $L)] rep $rep', d['value'], 'ms', d['ms_per_step'], 'conv', d['roofline']['achieved'], {n: (v['ms_per_step'], v['tflops']) for n, v in k.items()})"
  done
done
if [ -n "$KB" ]; then
  for L in $A $B; do
    echo "== kbench $(basename $L)"; CRNN_HIP_LIB=$PWD/$L timeout -k 10 100 python -u tools/kbench.py --iters 20 2>&1 | grep -v amdgpu
  done
fi
