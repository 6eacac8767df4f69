#!/bin/bash
# persistent-LSTM diagnostics: parity tests + in-kernel phase stamps
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "bilstm or handoff" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lstm.log 2>&1 || { tail -40 gpurun_out/pytest_lstm.log; exit 1; }
tail -2 gpurun_out/pytest_lstm.log
timeout -k 10 120 python -u tools/lstm_stamps.py > gpurun_out/stamps.log 2>&1; cat gpurun_out/stamps.log
timeout -k 10 120 python -u tools/lstm_stamps.py 64 64 768 > gpurun_out/stamps_long.log 2>&1; cat gpurun_out/stamps_long.log
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2>gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('VALUE', d['value'], 'ms', d['ms_per_step'], {k: v.get('us_per_timestep') for k, v in d['roofline_lstm'].items() if isinstance(v, dict)})"
fi
