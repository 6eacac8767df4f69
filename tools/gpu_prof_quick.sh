#!/bin/bash
# kernel-time profile of a short bench run: KTAG names the output, GREP filters the printed kernels
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${KTAG:-q} -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BARGS} > gpurun_out/prof_q.json 2> gpurun_out/prof_q.err || { tail -20 gpurun_out/prof_q.err; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_${KTAG:-q}/run_results.db 7 | head -45
