#!/bin/bash
# the GPU suite once more on the closing tree (a second box): stability of the co-scheduled determinism tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r05z8_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r05z8_pytest.log; grep -E "^FAILED" gpurun_out/r05z8_pytest.log | head; exit $rc
