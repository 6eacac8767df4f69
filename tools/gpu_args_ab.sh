#!/bin/bash
# In-box A/B of bench.py argument variants (same box, alternating order).
#   ARGAB="--kernel-timing all;--kernel-timing off" bash tools/gpu_args_ab.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
IFS=';' read -ra VARS <<< "$ARGAB"
for rep in $(seq 1 ${REPS:-2}); do
  for v in "${VARS[@]}"; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 $v > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed ($v)"; tail -20 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); k=d['kernels']; print('[$v] rep $rep', d['value'], 'ms', d['ms_per_step'], 'conv', d['roofline']['achieved'], {n: (v['ms_per_step'], v['tflops']) for n, v in k.items()})"
  done
done
