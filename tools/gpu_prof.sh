#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench command -> markdown summary (profiles/)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:?}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub ${BENCH_ARGS} > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof.err || { tail -20 gpurun_out/${T}_prof.err; exit 1; }
db=$(find gpurun_out/prof_$T -name "*.db" | head -1)
python tools/prof_summary.py --md "$db" 13 "${T} — rocprofv3 --kernel-trace --stats of \`python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub ${BENCH_ARGS}\` (13 traced steps)" > gpurun_out/${T}_summary.md
head -60 gpurun_out/${T}_summary.md
find gpurun_out/prof_$T -name "*stats*"
