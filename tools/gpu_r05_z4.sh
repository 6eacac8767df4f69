#!/bin/bash
# r05z4: BiLSTM weight gradients on the 4-wave GEMM form too (CRNN_OPT_GEMM4W mask 2 | 8 = 10): tests, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv or dgrad or bilstm" > gpurun_out/r05z4_test.log 2>&1
tail -3 gpurun_out/r05z4_test.log
GEMMBENCH_VENDOR= step timeout -k 10 200 python -u tools/gemmbench.py 14=2,10,2,10 > gpurun_out/r05z4_gemmbench.log 2>&1
grep -E "lstm wgrad|dwih|dwhh" gpurun_out/r05z4_gemmbench.log
for o in 2 10 2 10; do
  CRNN_OPTS="14=$o" step timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub > gpurun_out/r05z4_bench_f$o.json 2> gpurun_out/r05z4_bench_f$o.err
  python -c "import json;d=json.load(open('gpurun_out/r05z4_bench_f$o.json'));print('gemm4w $o', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
