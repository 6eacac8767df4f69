#!/bin/bash
# Alternating same-box A/B of bench.py lines under CRNN_OPTS variants:
#   gpurun -- 'TAG=x VARIANTS="6=1 6=3 14=0 default" ROUNDS=2 bash tools/bench_ab.sh'
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/${TAG:-ab}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    opts=$v; [ "$v" = "default" ] && opts=""
    CRNN_OPTS=$opts timeout -k 10 300 python -u bench.py --no-sub --no-cpu-baseline $BENCH_ARGS > ${O}_${v}_r$r.json 2>> ${O}_ab.err \
      || { tail -20 ${O}_ab.err; exit 1; }
    python -c "import json; d=json.load(open('${O}_${v}_r$r.json')); l=d['roofline_lstm']; print('$v r$r', d['value'], d['ms_per_step'], 'conv', d['roofline']['frac'], {k: d['kernels'][k]['tflops'] for k in d['kernels']}, 'lstm', l['lstm_fwd']['us_per_timestep'], l['lstm_bwd']['us_per_timestep'])" | tee -a ${O}_ab.log
  done
done
