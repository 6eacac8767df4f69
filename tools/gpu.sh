#!/bin/bash
# The one GPU runner:   gpurun --timeout S -- 'TAG=r06x bash tools/gpu.sh STEP [STEP ...]'
# Each step runs under its own time limit; the first failing step ends the call (nothing retries).
# Outputs: gpurun_out/<TAG>_<step>.*  (copy what is judged into profiles/).
# Steps:
#   tests      python -m pytest tests -m gpu  (PYTEST_K selects with -k; PYTEST_T = timeout, default 1000 s)
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py $BENCH_ARGS (default: the driver's line, sub-measurements and CPU baseline included)
#   modes      bench lines --path engine, --mode infer, --config long, --mode attn_train (no CPU baseline)
#   prof       rocprofv3 --kernel-trace --stats of bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub
#              $BENCH_ARGS + a markdown summary (tools/prof_summary.py)
#   pmc        PMC passes over bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-sub (FETCH_SIZE; WRITE_SIZE;
#              MFMA busy + GUI active), one counter group per run, kernel-trace only -> <TAG>_pmc_traffic.json,
#              also copied to profiles/ (stamped with this tree's source hash, read by bench.py)
#   dp         N-rank (N=${N:-2}) one-device rehearsal of python bench.py --gpus N (gloo over GPU tensors, per-step
#              BiLSTM launches)
#   py:SCRIPT  python tools/SCRIPT $PY_ARGS (PY_T = timeout, default 300 s)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-run}
mkdir -p gpurun_out
O=gpurun_out/$T
BENCH_PROF="--steps 10 --warmup 3 --no-cpu-baseline --no-sub"

for step in "$@"; do
  case "$step" in
  tests)
    sel=(); [ -n "$PYTEST_K" ] && sel=(-k "$PYTEST_K")
    timeout -k 10 ${PYTEST_T:-1000} python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread $PYTEST_EXTRA \
      "${sel[@]}" > ${O}_pytest.log 2>&1 || { grep -E "^FAILED|Error" ${O}_pytest.log | head -20; tail -30 ${O}_pytest.log; exit 1; }
    tail -2 ${O}_pytest.log ;;
  smoke)
    timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 \
      || { cat ${O}_smoke.log; exit 1; }
    tail -1 ${O}_smoke.log ;;
  bench)
    timeout -k 10 600 python -u bench.py $BENCH_ARGS > ${O}_bench.json 2> ${O}_bench.err || { tail -20 ${O}_bench.err; exit 1; }
    cut -c1-1500 ${O}_bench.json ;;
  modes)
    for m in "--path engine" "--mode infer" "--config long" "--mode attn_train"; do
      f=$(echo "$m" | tr -d ' -')
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-sub $m > ${O}_bench_$f.json 2>> ${O}_bench.err \
        || { tail -20 ${O}_bench.err; exit 1; }
      python -c "import json; d=json.load(open('${O}_bench_$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('roofline', {}).get('frac'))"
    done ;;
  prof)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_prof -o run -- python3 bench.py $BENCH_PROF $BENCH_ARGS \
      > ${O}_prof_bench.json 2> ${O}_prof.err || { tail -20 ${O}_prof.err; exit 1; }
    db=$(find ${O}_prof -name "*.db" | head -1)
    python tools/prof_summary.py --md "$db" 13 "${T} — rocprofv3 --kernel-trace --stats of \`python bench.py $BENCH_PROF $BENCH_ARGS\` (13 traced steps)" > ${O}_summary.md
    head -40 ${O}_summary.md ;;
  pmc)
    i=0
    for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
      i=$((i+1))
      timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d ${O}_pmc_$i -o run -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-sub > ${O}_pmc_$i.log 2>&1 \
        || { echo "pmc pass $i ($C) failed"; tail -20 ${O}_pmc_$i.log; exit 1; }
    done
    python tools/pmc_traffic.py ${O}_pmc_1 ${O}_pmc_2 ${O}_pmc_3 > ${O}_pmc_traffic.json || exit 1
    cp ${O}_pmc_traffic.json profiles/${T}_pmc_traffic.json
    python -c "import json; d=json.load(open('${O}_pmc_traffic.json')); print({k: (v.get('hbm_bytes_per_launch'), v.get('mfma_busy_frac')) for k, v in d.items() if isinstance(v, dict)})" ;;
  dp)
    CRNN_SHARE_DEVICE=1 CRNN_DIST_BACKEND=gloo CRNN_LSTM_PER_STEP=1 timeout -k 10 300 python -u bench.py --gpus ${N:-2} \
      --steps 3 --warmup 1 --batch ${BATCH:-64} --no-sub > ${O}_dp${N:-2}.json 2> ${O}_dp${N:-2}.err \
      || { tail -30 ${O}_dp${N:-2}.err; exit 1; }
    cut -c1-600 ${O}_dp${N:-2}.json ;;
  py:*)
    s=${step#py:}
    timeout -k 10 ${PY_T:-300} python -u tools/$s $PY_ARGS > ${O}_${s%.py}.log 2>&1 || { tail -30 ${O}_${s%.py}.log; exit 1; }
    tail -${PY_TAIL:-25} ${O}_${s%.py}.log ;;
  *)
    echo "unknown step $step"; exit 2 ;;
  esac
done
