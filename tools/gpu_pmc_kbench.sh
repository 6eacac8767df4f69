#!/bin/bash
# one PMC pass over a per-layer conv microbench: PMC="counters" KB_ARGS="--layer 1 --only fwd"
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d gpurun_out/pmck -o run -- python3 tools/kbench.py --iters 3 $KB_ARGS > gpurun_out/pmck.log 2>&1 || { echo "pmc pass failed"; tail -20 gpurun_out/pmck.log; exit 1; }
f=$(find gpurun_out/pmck -name "run_counter_collection.csv" | head -1)
python3 tools/pmc_kernels.py $(dirname $f) ${SUB}
