#!/bin/bash
# HBM traffic per conv kernel per layer: FETCH_SIZE / WRITE_SIZE passes over tools/kbench.py
# (--iters 2); summarize with tools/pmc_kbench_summary.py gpurun_out/pmck_F gpurun_out/pmck_W
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmck_${C:0:1} -o run -- python3 tools/kbench.py --iters 2 > gpurun_out/pmck_${C:0:1}.log 2>&1 || { tail -5 gpurun_out/pmck_${C:0:1}.log; exit 1; }
done
