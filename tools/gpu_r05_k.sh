#!/bin/bash
# r05k: packed-fp32 hypothesis — the co-residency probe (both models per-step BiLSTM) with the default library
# and with a build whose device code has no packed fp32 VALU ops (v_pk_fma/add/mul_f32)
set -o pipefail
o=gpurun_out/r05k
mkdir -p $o
step() {
  local log=$1; shift
  "$@" > $o/$log 2>&1
  local rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ge 124 ]; then tail -n 20 $o/$log; exit $rc; fi
  return 0
}
step cohab_00_default_a.log env COHAB_PROBE=1 timeout -k 10 300 python -u tools/cohab_model.py 100 0 0 model
step cohab_00_nopk_a.log env CRNN_HIP_LIB=$PWD/rcnn-ocr_amd/crnn_hip/libcrnn_hip_nopk.so COHAB_PROBE=1 timeout -k 10 300 python -u tools/cohab_model.py 100 0 0 model
step cohab_00_default_b.log env COHAB_PROBE=1 timeout -k 10 300 python -u tools/cohab_model.py 100 0 0 model
step cohab_00_nopk_b.log env CRNN_HIP_LIB=$PWD/rcnn-ocr_amd/crnn_hip/libcrnn_hip_nopk.so COHAB_PROBE=1 timeout -k 10 300 python -u tools/cohab_model.py 100 0 0 model
for f in $o/*.log; do echo "$f: $(grep SUMMARY $f)"; done
exit 0
