#!/bin/bash
# the other BASELINE configs as bench modes: configs[1] inference, configs[4] long lines
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --mode infer --steps 20 --warmup 3 > gpurun_out/bench_infer.json 2> gpurun_out/bench_infer.err || { tail -20 gpurun_out/bench_infer.err; exit 1; }
cut -c1-1200 gpurun_out/bench_infer.json
timeout -k 10 400 python -u bench.py --config long --steps 5 --warmup 2 --cpu-sample 4 --cpu-steps 2 > gpurun_out/bench_long.json 2> gpurun_out/bench_long.err || { tail -20 gpurun_out/bench_long.err; exit 1; }
cut -c1-1500 gpurun_out/bench_long.json
