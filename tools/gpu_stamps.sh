#!/bin/bash
# persistent-LSTM diagnostics: parity tests + in-kernel phase stamps
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k bilstm -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lstm.log 2>&1 || { tail -40 gpurun_out/pytest_lstm.log; exit 1; }
tail -2 gpurun_out/pytest_lstm.log
timeout -k 10 120 python -u tools/lstm_stamps.py > gpurun_out/stamps.log 2>&1; cat gpurun_out/stamps.log
