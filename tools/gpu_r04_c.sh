#!/bin/bash
# r04 batch c: same-box A/B of the conv wgrad slab reduce on a side stream (0/1 alternating), bench
# default lines; then the determinism + kernel checks of batch a on this tree
mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > gpurun_out/r04c_$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
for r in 1 2; do
  for v in 0 1; do
    CRNN_WGRAD_REDUCE_STREAM=$v step bench_rs${v}_$r timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 30 --warmup 5
  done
done
step det timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_determinism.py
