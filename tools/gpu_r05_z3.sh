#!/bin/bash
# r05z3: BN-fused conv input gradients on the 4-wave GEMM form too (CRNN_OPT_GEMM4W = 3): tests, kbench, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv or dgrad" > gpurun_out/r05z3_test.log 2>&1
tail -3 gpurun_out/r05z3_test.log
for o in 2 3 2 3; do
  CRNN_OPTS="14=$o" step timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub > gpurun_out/r05z3_bench_f$o.json 2> gpurun_out/r05z3_bench_f$o.err
  python -c "import json;d=json.load(open('gpurun_out/r05z3_bench_f$o.json'));print('gemm4w $o', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms_per_step'])"
done
