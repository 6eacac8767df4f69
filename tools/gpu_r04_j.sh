#!/bin/bash
# r04 batch j: conv-only checker next to a bench.py load process (bf16, then fp32) on the same GPU
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
one() {  # name, extra bench args
  timeout -k 10 200 python -u bench.py --steps 100000 --warmup 2 --batch 128 --no-cpu-baseline --kernel-timing off $2 \
      > gpurun_out/r04j_load_$1.log 2>&1 &
  local LP=$!
  sleep 30
  timeout -k 10 120 python -u tools/conv_only_check.py 70 > gpurun_out/r04j_conv_$1.log 2>&1
  local rc=$?
  kill $LP; wait $LP
  echo "$1 checker rc=$rc"; tail -1 gpurun_out/r04j_conv_$1.log
  [ $rc -eq 0 ] || exit $rc
}
one bf16 "" && one fp32 "--dtype fp32"
