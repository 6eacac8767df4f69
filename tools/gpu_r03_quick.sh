#!/bin/bash
# quick loop: selected GPU tests, the train bench, and a rocprof kernel summary of it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:?}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${PYTEST_PATHS:-tests/test_gpu_kernels.py} -m gpu -x -q -rP --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/${T}_pytest.log | head; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels'], d['roofline_lstm']['lstm_fwd']['frac'], d['roofline_lstm']['lstm_bwd']['frac'])"
[ -n "$NO_PROF" ] && exit 0
TAG=$T bash tools/gpu_prof.sh > /dev/null 2>&1 || { echo "prof failed"; exit 1; }
head -40 gpurun_out/${T}_summary.md
