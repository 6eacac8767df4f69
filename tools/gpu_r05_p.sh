#!/bin/bash
# r05p: persistent BiLSTM prologue (step-0 inputs issued ahead of the W_hh slice loads) + entry stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "lstm_seq" > gpurun_out/r05p_test.log 2>&1
tail -3 gpurun_out/r05p_test.log
STAMPS_SAVE_AB=1 step timeout -k 10 200 python -u tools/lstm_stamps.py 256 32 512 > gpurun_out/r05p_stamps.log 2>&1
cat gpurun_out/r05p_stamps.log
STAMPS_SAVE_AB=1 step timeout -k 10 200 python -u tools/lstm_stamps.py 64 64 768 > gpurun_out/r05p_stamps_long.log 2>&1
cat gpurun_out/r05p_stamps_long.log
step timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub > gpurun_out/r05p_bench.json 2> gpurun_out/r05p_bench.err
python -c "import json;d=json.load(open('gpurun_out/r05p_bench.json'));print(d['value'], d['ms_per_step'], d['roofline_lstm'])"
