#!/bin/bash
# quick iteration: selected GPU tests (PYTEST_K) + full GPU suite + bench (+ optional rocprof)
cd $GRAFT_REPO_ROOT
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -k "$PYTEST_K" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { tail -40 gpurun_out/pytest_sel.log; exit 1; }
  tail -2 gpurun_out/pytest_sel.log
fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2>gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('VALUE', d['value'], 'ms', d['ms_per_step'], 'conv', d['roofline']['achieved'], {k: v.get('us_per_timestep') for k, v in d['roofline_lstm'].items() if isinstance(v, dict)})"
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$PROF -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { tail -30 gpurun_out/prof.err; exit 1; }
  echo "profiled"
fi
