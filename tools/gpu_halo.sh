#!/bin/bash
# halo conv: parity tests, per-layer A/B against the GEMM path, bench
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "conv" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_halo.log 2>&1 || { tail -40 gpurun_out/pytest_halo.log; exit 1; }
tail -2 gpurun_out/pytest_halo.log
timeout -k 10 200 python -u tools/kbench.py --layer 1 --opt 5=1,0 > gpurun_out/kbench_halo.log 2>&1; grep -v amdgpu gpurun_out/kbench_halo.log
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2>gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('VALUE', d['value'], 'ms', d['ms_per_step'], d['roofline']['achieved'])"
fi
