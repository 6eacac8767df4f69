#!/bin/bash
# r05s: 16-B row stores for the linear / BiLSTM projection epilogue (CRNN_OPT_LINEAR_ROW8): parity, GEMM A/B, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "row8 or gemm_nt" > gpurun_out/r05s_test.log 2>&1
tail -3 gpurun_out/r05s_test.log
GEMMBENCH_VENDOR=1 step timeout -k 10 200 python -u tools/gemmbench.py 20=0,1,0,1 > gpurun_out/r05s_gemmbench.log 2>&1
cat gpurun_out/r05s_gemmbench.log
for o in 0 1 0 1; do
  CRNN_OPTS="20=$o" step timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub > gpurun_out/r05s_bench_r$o.json 2> gpurun_out/r05s_bench_r$o.err
  python -c "import json;d=json.load(open('gpurun_out/r05s_bench_r$o.json'));print('row8 $o', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
