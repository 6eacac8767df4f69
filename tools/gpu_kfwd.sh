#!/bin/bash
# conv A/B: tests, per-layer conv microbench with option OPT (KEY=V0,V1), bench
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -k "conv or e2e" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { tail -30 gpurun_out/pytest_sel.log; exit 1; }
tail -1 gpurun_out/pytest_sel.log
timeout -k 10 300 python -u tools/kbench.py ${KB_ARGS} > gpurun_out/kbench.log 2>&1; grep -v amdgpu gpurun_out/kbench.log
bash tools/gpu_quick.sh
