#!/bin/bash
# torch-only checker process next to a bench.py load process on the same GPU
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 260 python -u bench.py --steps 6000 --warmup 5 --no-cpu-baseline --kernel-timing off > gpurun_out/r04h_load.log 2>&1 &
LP=$!
sleep 30
timeout -k 10 150 python -u tools/torch_only_check.py 90 > gpurun_out/r04h_torch_only.log 2>&1
rc=$?
wait $LP
echo "checker rc=$rc"
tail -3 gpurun_out/r04h_torch_only.log
exit $rc
