#!/bin/bash
# cohab probe with quantified first differences, then the resident-sentinel LDS probe (rewrite + shuffle checks)
set -o pipefail
COHAB_PROBE=1 timeout -k 10 200 python -u tools/cohab_model.py 24 1 0 model > gpurun_out/r05h_cohab_probe.log 2>&1 &&
timeout -k 10 400 python -u tools/lds_sentinel.py --rounds 6 --blocks 256 --iters 600 --launches 8 --lds 4096,16384 --mode 3 > gpurun_out/r05h_sentinel_resident.log 2>&1
rc=$?
grep -A1 "^iter" gpurun_out/r05h_cohab_probe.log | grep -B1 "SE chain" | cut -c1-900
grep SUMMARY gpurun_out/r05h_*.log
exit $rc
