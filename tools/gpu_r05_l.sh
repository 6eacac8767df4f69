#!/bin/bash
# r05l: cost of building without packed fp32 VALU ops — default vs no-packed library, alternating, one box
set -o pipefail
o=gpurun_out/r05l
mkdir -p $o
NOPK=$PWD/rcnn-ocr_amd/crnn_hip/libcrnn_hip_nopk.so
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub > $o/bench_pk_r$r.json 2> $o/bench_pk_r$r.err || exit $?
  CRNN_HIP_LIB=$NOPK timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub > $o/bench_nopk_r$r.json 2> $o/bench_nopk_r$r.err || exit $?
done
for f in $o/*.json; do python -c "
import json,sys; d=json.load(open('$f')); k=d['kernels']
print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], {n: v['ms_per_step'] for n, v in k.items()}, d['roofline_lstm']['lstm_fwd']['us_per_timestep'], d['roofline_lstm']['lstm_bwd']['us_per_timestep'])"; done
