#!/bin/bash
# in-process co-residency bisection (tools/cohab_model.py); one log per variant under gpurun_out/
set -o pipefail
o=gpurun_out/r05d
mkdir -p $o
t() { timeout -k 10 150 python -u tools/cohab_model.py "$@"; }
t 16 0 0 hog:256:65536:6000 > $o/hog64k_v0.log 2>&1 &&
t 16 1 0 hog:256:65536:6000 > $o/hog64k_v1.log 2>&1 &&
t 16 0 0 hog:1024:16384:6000 > $o/hog16k_v0.log 2>&1 &&
CRNN_OPTS=13=0 t 16 1 0 model > $o/model_v1_l2off.log 2>&1 &&
t 16 1 0 model > $o/model_v1.log 2>&1
rc=$?
grep -h SUMMARY $o/*.log
exit $rc
