#!/bin/bash
# r04 batch b: two-process determinism A/B (ticketed vs one-launch BN finalize), the DP tests with the
# exact bar, run_training world 2, the POOL_OUT wide-group kernel test. A test failure (rc 1) lets
# the next step run; any other status ends the script.
mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > gpurun_out/r04b_$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
for o in 1 0; do
  CRNN_DET_SET=17=$o step det_load_opt$o timeout -k 10 240 python -u tools/det_load.py 30
done
step dp timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_dp.py tests/test_train_dp.py
step pool timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "pool_mode or colsum or finalize"
step refmodel timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_refmodel.py tests/test_gpu_parity_bench.py -k "refmodel or train_step"
