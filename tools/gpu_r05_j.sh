#!/bin/bash
# r05j: co-residency statistics (100 iterations per configuration), quantified first differences
set -o pipefail
o=gpurun_out/r05j
mkdir -p $o
step() {
  local log=$1; shift
  "$@" > $o/$log 2>&1
  local rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ge 124 ]; then tail -n 20 $o/$log; exit $rc; fi
  return 0
}
step cohab_10.log env COHAB_PROBE=1 timeout -k 10 300 python -u tools/cohab_model.py 100 1 0 model
step cohab_00.log env COHAB_PROBE=1 timeout -k 10 300 python -u tools/cohab_model.py 100 0 0 model
grep -h SUMMARY $o/*.log
grep -h -A1 "^iter" $o/*.log | grep "SE chain" | cut -c1-700
exit 0
