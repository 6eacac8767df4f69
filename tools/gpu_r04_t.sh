#!/bin/bash
# r04 batch t: BiLSTM dx on the 256-row kernel — LSTM kernel tests, bench A/B of option 19 (alternated)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 240 --timeout-method thread -k "lstm or bilstm or finalize" > gpurun_out/r04t_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04t_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04t_tests.log | head -20; exit 1; }
for r in 1 2; do
  for v in 0 1; do
    CRNN_OPTS=19=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/r04t_bench_o${v}_r${r}.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r04t_bench_o${v}_r${r}.json')); print('opt19=$v rep $r', d['value'], d['ms_per_step'])"
  done
done
