#!/bin/bash
# r03x: GPU tests, API + engine bench, rocprof trace (gap analysis of the API step)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r03x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${PYTEST_PATHS:-tests} -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/${T}_pytest.log | head -20; exit 1; }
for p in api engine api; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --path $p > gpurun_out/${T}_bench_$p.json 2>> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_bench_$p.json')); print('$p', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_lstm']['lstm_fwd']['frac'], d['roofline_lstm']['lstm_bwd']['frac'])"
done
TAG=$T bash tools/gpu_prof.sh > /dev/null 2>&1 || { echo "prof failed"; tail gpurun_out/${T}_prof.err; exit 1; }
python tools/step_gaps.py gpurun_out/prof_$T/run_results.db
