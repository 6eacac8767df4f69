#!/bin/bash
# r04 batch n: full GPU suite with the W-halo kernel on, then bench A/B of option 18 in alternation
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04n_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r04n_pytest.log; grep -E "^FAILED" gpurun_out/r04n_pytest.log | head; [ $rc -le 1 ] || exit 1
for r in 1 2; do
  for v in 0 1; do
    CRNN_OPTS=18=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/r04n_bench_o${v}_r${r}.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r04n_bench_o${v}_r${r}.json')); print('opt18=$v rep $r', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels'])"
  done
done
