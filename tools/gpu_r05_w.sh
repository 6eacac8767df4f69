#!/bin/bash
# r05w: stem input conv weight gradient at one workgroup per band (CRNN_OPT_HALO_WG2): parity, kernel A/B, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "halo" > gpurun_out/r05w_test.log 2>&1
tail -3 gpurun_out/r05w_test.log
step timeout -k 10 200 python -u tools/halo_ab.py 22 > gpurun_out/r05w_halo_ab.log 2>&1
cat gpurun_out/r05w_halo_ab.log
for o in 0 1 0 1; do
  CRNN_OPTS="22=$o" step timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub > gpurun_out/r05w_bench_g$o.json 2> gpurun_out/r05w_bench_g$o.err
  python -c "import json;d=json.load(open('gpurun_out/r05w_bench_g$o.json'));print('wg2 $o', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
