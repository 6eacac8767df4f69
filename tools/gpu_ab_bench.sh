#!/bin/bash
# In-box A/B of bench.py under CRNN_OPTS variants (same box, alternating order), plus selected tests.
#   AB="10=0;10=1" PYTEST_K="conv" bash tools/gpu_ab_bench.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -k "$PYTEST_K" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { tail -40 gpurun_out/pytest_sel.log; exit 1; }
  tail -2 gpurun_out/pytest_sel.log
fi
IFS=';' read -ra VARS <<< "$AB"
for rep in 1 2; do
  for v in "${VARS[@]}"; do
    CRNN_OPTS="$v" timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed ($v)"; tail -20 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); k=d['kernels']; print('[$v] rep $rep', d['value'], 'ms', d['ms_per_step'], 'conv', d['roofline']['achieved'], {n: (v['ms_per_step'], v['tflops']) for n, v in k.items()}, {n: v.get('us_per_timestep') for n, v in d['roofline_lstm'].items() if isinstance(v, dict)})"
  done
done
