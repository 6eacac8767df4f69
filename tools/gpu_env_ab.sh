#!/bin/bash
# In-box A/B of bench.py under environment-variable variants (same box, alternating order), plus
# selected GPU tests first.
#   ENVAB="CRNN_WGRAD_STREAM=0;CRNN_WGRAD_STREAM=1" PYTEST_K="side_stream" BARGS="--mode train" bash tools/gpu_env_ab.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -k "$PYTEST_K" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { tail -40 gpurun_out/pytest_sel.log; exit 1; }
  tail -2 gpurun_out/pytest_sel.log
fi
IFS=';' read -ra VARS <<< "$ENVAB"
for rep in $(seq 1 ${REPS:-2}); do
  for v in "${VARS[@]}"; do
    env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 ${BARGS} > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed ($v)"; tail -20 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); k=d['kernels']; print('[$v] rep $rep', d['value'], 'ms', d['ms_per_step'], 'conv', d['roofline']['achieved'], {n: (v['ms_per_step'], v['tflops']) for n, v in k.items()}, {n: v.get('us_per_timestep') for n, v in (d.get('roofline_lstm') or {}).items() if isinstance(v, dict)})"
  done
done
