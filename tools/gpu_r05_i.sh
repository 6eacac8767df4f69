#!/bin/bash
# r05i: the pipelined BiLSTM forward (parity test + in-process A/B), the co-residency probes, the refmodel trace
set -o pipefail
o=gpurun_out/r05i
mkdir -p $o
# a step that times out, aborts or faults (rc >= 124) ends the call; an ordinary failure (assertion, python
# error) is reported and the next step runs
step() {
  local log=$1; shift
  "$@" > $o/$log 2>&1
  local rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ge 124 ]; then
    tail -n 20 $o/$log
    exit $rc
  fi
  return 0
}
step pipe_tests.log timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -s --timeout 120 --timeout-method thread -k "pipelined or handoff_forms or l2_handoff or bwd_forms"
step pipe_ab_cfg2.log timeout -k 10 120 python -u tools/lstm_ab.py 19=0,3
step pipe_ab_long.log timeout -k 10 120 python -u tools/lstm_ab.py 19=0,3 64 128 768
step cohab_probe.log env COHAB_PROBE=1 timeout -k 10 200 python -u tools/cohab_model.py 24 1 0 model
step cohab_probe_hostkernarg.log env HIP_FORCE_DEV_KERNARG=0 COHAB_PROBE=1 timeout -k 10 200 python -u tools/cohab_model.py 24 1 0 model
step refmodel_trace.log timeout -k 10 200 python -u tools/refmodel_trace.py
step sentinel_resident.log timeout -k 10 400 python -u tools/lds_sentinel.py --rounds 6 --blocks 256 --iters 600 --launches 8 --lds 4096,16384 --mode 3
grep -E "passed|failed" $o/pipe_tests.log | tail -n 2
grep "pipe vs" $o/pipe_tests.log | head -n 12
cat $o/pipe_ab_*.log
grep -A1 "^iter" $o/cohab_probe.log | grep -B1 "SE chain" | cut -c1-900
grep -h SUMMARY $o/*.log
tail -n 6 $o/refmodel_trace.log
exit 0
