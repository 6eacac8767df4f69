#!/bin/bash
# r05o: deferred saved-forward stores in the persistent BiLSTM forward (CRNN_OPT_LSTM_DEFER):
# parity (bit-identical to the other hand-off forms) + per-step stamps A/B + bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "handoff_forms_agree" > gpurun_out/r05o_test.log 2>&1
tail -3 gpurun_out/r05o_test.log
STAMPS_SAVE_AB=1 step timeout -k 10 200 python -u tools/lstm_stamps.py 256 32 512 > gpurun_out/r05o_stamps.log 2>&1
cat gpurun_out/r05o_stamps.log
for d in 0 1 0 1; do
  CRNN_OPTS="20=$d" step timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sub > gpurun_out/r05o_bench_d$d.json 2> gpurun_out/r05o_bench_d$d.err
  python -c "import json;d=json.load(open('gpurun_out/r05o_bench_d$d.json'));print('defer $d', d['value'], d['ms_per_step'], d['roofline_lstm'])"
done
