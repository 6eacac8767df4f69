#!/bin/bash
# r04: two-process determinism (tools/det_load.py: a bench.py process loads the GPU) with the
# r03 ticketed BN finalize (option 17 = 1) and the one-launch finalize (17 = 0)
mkdir -p gpurun_out
for o in 1 0; do
  CRNN_DET_SET=17=$o timeout -k 10 240 python -u tools/det_load.py 30 > gpurun_out/r04b_det_load_opt$o.log 2>&1
  rc=$?; echo "det_load opt $o rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
