#!/bin/bash
# GPU iteration script: LSTM kernel tests, full GPU suite, bench (new vs per-step LSTM).
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k bilstm -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_lstm.log 2>&1 || { tail -40 gpurun_out/pytest_lstm.log; exit 1; }
tail -3 gpurun_out/pytest_lstm.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2>gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
CRNN_LSTM_PER_STEP=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_perstep.json 2>gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench_perstep.json
