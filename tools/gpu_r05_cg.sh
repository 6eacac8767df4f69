#!/bin/bash
# r05cg: strided dgrad class groups on 256 x 256 tiles (CRNN_OPT_DGRAD_GROUP = 2): parity, kbench, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "class_group or dgrad" > gpurun_out/r05cg_test.log 2>&1
tail -3 gpurun_out/r05cg_test.log
step timeout -k 10 240 python -u tools/kbench.py --iters 10 --only dgrad --opt 16=1,2,1,2 > gpurun_out/r05cg_kbench.log 2>&1
grep -E "b0.c1|b3.c1|co0" gpurun_out/r05cg_kbench.log
for o in 1 2 1 2; do
  CRNN_OPTS="16=$o" step timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub > gpurun_out/r05cg_bench_g$o.json 2> gpurun_out/r05cg_bench_g$o.err
  python -c "import json;d=json.load(open('gpurun_out/r05cg_bench_g$o.json'));print('dgrad_group $o', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
