#!/bin/bash
# r04 batch l: W-halo A image conv kernel — parity tests, per-layer A/B (option 18 = 0 / 1 / 2)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 240 --timeout-method thread -k "conv" > gpurun_out/r04l_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04l_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04l_tests.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/kbench.py --only fwd --opt 18=0,1 > gpurun_out/r04l_kbench_fwd.log 2>&1 || exit 1
cat gpurun_out/r04l_kbench_fwd.log | grep -v "^$" | tail -40
timeout -k 10 300 python -u tools/kbench.py --only dgrad --opt 18=0,1 > gpurun_out/r04l_kbench_dgrad.log 2>&1 || exit 1
grep -E "b[0-9]+\.c2|b3.c2|sum" gpurun_out/r04l_kbench_dgrad.log | tail -20
