#!/bin/bash
# wgrad A/B (fast per-tile pixel decode vs per-lane decode) + conv parity tests
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "conv" -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_conv.log 2>&1 || { tail -30 gpurun_out/pt_conv.log; exit 1; }
tail -2 gpurun_out/pt_conv.log
timeout -k 10 200 python -u tools/kbench.py --iters 20 --only wgrad --opt 8=0,1 > gpurun_out/kb_wfast.log 2>&1 || { tail -20 gpurun_out/kb_wfast.log; exit 1; }
cat gpurun_out/kb_wfast.log
