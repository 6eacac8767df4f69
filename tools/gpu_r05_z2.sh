#!/bin/bash
# r05z2: conv weight gradients on the 4-wave GEMM (CRNN_OPT_GEMM4W = 2) and the 256 x 128 wgrad tile at Kp = 256:
# kernel tests, per-layer kbench A/B, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv" > gpurun_out/r05z2_test.log 2>&1
tail -3 gpurun_out/r05z2_test.log
step timeout -k 10 240 python -u tools/kbench.py --iters 10 --only wgrad --opt 14=2,0,2,0 > gpurun_out/r05z2_kbench.log 2>&1
grep -v amdgpu.ids gpurun_out/r05z2_kbench.log
for o in 0 2 0 2; do
  CRNN_OPTS="14=$o" step timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub > gpurun_out/r05z2_bench_f$o.json 2> gpurun_out/r05z2_bench_f$o.err
  python -c "import json;d=json.load(open('gpurun_out/r05z2_bench_f$o.json'));print('gemm4w $o', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
