#!/bin/bash
# r04 batch k: BN finalize rewrite — kernel tests, under-load determinism, finalize microbench, bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_determinism.py tests/test_gpu_parity_bench.py -q -x --timeout 240 --timeout-method thread -k "finalize or bn or determinism or bench_selection" > gpurun_out/r04k_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04k_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_refmodel.py -q --timeout 240 --timeout-method thread -s > gpurun_out/r04k_refmodel.log 2>&1; grep -E "fp32:|bf16:|passed|failed" gpurun_out/r04k_refmodel.log
timeout -k 10 120 python -u tools/bnbench.py > gpurun_out/r04k_bnbench.log 2>&1 || exit 1
cat gpurun_out/r04k_bnbench.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r04k_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], {k: (v['us_per_sweep'], v['frac']) for k, v in d['roofline_lstm'].items() if isinstance(v, dict)})"
TAG=r04k bash tools/gpu_prof.sh > /dev/null 2>&1 || exit 1
grep -E "fin_one|lstm_seq" gpurun_out/r04k_summary.md
