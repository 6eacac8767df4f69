#!/bin/bash
# r04 batch r: tile-group size A/B (GEMM_GROUP_M 8 default vs 4 vs 16 builds), alternated, same box
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/rcnn-ocr_amd/crnn_hip
for r in 1 2; do
  for v in g8 g4 g16; do
    lib=$L/libcrnn_hip_$v.so; [ $v = g8 ] && lib=$L/libcrnn_hip.so
    CRNN_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/r04r_bench_${v}_r${r}.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r04r_bench_${v}_r${r}.json')); print('$v rep $r', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
  done
done
