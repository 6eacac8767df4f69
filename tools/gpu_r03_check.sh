#!/bin/bash
# r03: GPU test suite (incl. the bench-selection parity tests), smoke, train bench on the API path
# and on the engine path (A/B of the drop-in API's overhead), inference bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r03}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${PYTEST_PATHS:-tests} -m gpu -x -v -rP --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/${T}_pytest.log | head -20; exit 1; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { cat gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/${T}_bench_api.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --path engine > gpurun_out/${T}_bench_engine.json 2>> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/${T}_bench_api2.json 2>> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --mode infer --no-cpu-baseline > gpurun_out/${T}_bench_infer.json 2>> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
for f in api engine api2 infer; do python -c "import json,sys; d=json.load(open('gpurun_out/${T}_bench_$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('roofline_lstm',{}).get('lstm_fwd',{}).get('frac'))"; done
