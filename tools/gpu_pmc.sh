#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only; MI355X_MICROARCH.md "HBM" / PMC slots):
# FETCH_SIZE, WRITE_SIZE, MFMA busy + GUI active, over a short bench run.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ARGS="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-sub"
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_$i -o run -- python3 $ARGS > gpurun_out/pmc_$i.log 2>&1 || { echo "pass $i ($C) failed"; tail -20 gpurun_out/pmc_$i.log; exit 1; }
  echo "pass $i ($C) ok"
done
find gpurun_out/pmc_* -name "*.csv" | head -20
