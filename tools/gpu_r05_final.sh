#!/bin/bash
# r05 closing measurements on one box: full GPU test suite, smoke, the default bench line (train,
# API path), engine-path and other-config bench lines, rocprof kernel summary, PMC traffic passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r05z}
mkdir -p gpurun_out
if [ "$PART" != "bench" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log; grep -E "^FAILED" gpurun_out/${T}_pytest.log | head -20; [ $rc -le 1 ] || exit 1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { cat gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
[ "$PART" = "tests" ] && exit 0
fi
# PMC traffic first, stamped with this tree's source hash and placed where bench.py looks for it, so the
# bench lines below carry it (the driver's round-end bench runs on the committed copy)
bash tools/gpu_pmc.sh > gpurun_out/${T}_pmc.log 2>&1 || { tail gpurun_out/${T}_pmc.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc_1 gpurun_out/pmc_2 gpurun_out/pmc_3 > gpurun_out/${T}_pmc_traffic.json || exit 1
cp gpurun_out/${T}_pmc_traffic.json profiles/${T}_pmc_traffic.json
python -c "import json; d=json.load(open('gpurun_out/${T}_pmc_traffic.json')); print({k: (v.get('hbm_bytes_per_launch'), v.get('mfma_busy_frac')) for k, v in d.items() if isinstance(v, dict)})"
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
for m in "--path engine" "--mode infer" "--config long" "--mode attn_train"; do
  f=$(echo "$m" | tr -d ' -')
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-sub $m > gpurun_out/${T}_bench_$f.json 2>> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
done
for f in gpurun_out/${T}_bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))"; done
TAG=$T bash tools/gpu_prof.sh > /dev/null 2>&1 || { echo "prof failed"; tail gpurun_out/${T}_prof.err; exit 1; }
