#!/bin/bash
# r04 batch p: conv kernel tests + bench A/B of the W-halo option (alternating, same box)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_determinism.py -q -x --timeout 240 --timeout-method thread -k "conv or determinism" > gpurun_out/r04p_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04p_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04p_tests.log | head -20; exit 1; }
for r in 1 2; do
  for v in 0 1; do
    CRNN_OPTS=18=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/r04p_bench_o${v}_r${r}.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r04p_bench_o${v}_r${r}.json')); print('opt18=$v rep $r', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
  done
done
