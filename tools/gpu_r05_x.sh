#!/bin/bash
# r05x: data-parallel rehearsal of bench.py on one GPU (gloo), 2 and 4 ranks: the DP fields of the line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=2 bash tools/gpu_dp_rehearsal.sh || exit 1
N=4 bash tools/gpu_dp_rehearsal.sh || exit 1
python - <<'PY'
import json
for n in (2, 4):
    d = json.load(open(f"gpurun_out/dp{n}.json"))
    print(n, d["value"], d["ms_per_step"], {k: v for k, v in d.get("dp", {}).items() if k != "exposed_note"})
PY
