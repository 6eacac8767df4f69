#!/bin/bash
# the headline bench line plus every other bench mode on one box (BASELINE configs[1], [4])
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err || { tail -20 gpurun_out/bench_train.err; exit 1; }
cut -c1-600 gpurun_out/bench_train.json
for m in infer attn attn_train preprocess; do
  timeout -k 10 300 python -u bench.py --mode $m --steps 20 --warmup 3 > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err || { tail -20 gpurun_out/bench_$m.err; exit 1; }
  cut -c1-300 gpurun_out/bench_$m.json
done
timeout -k 10 400 python -u bench.py --config long --steps 5 --warmup 2 --cpu-sample 4 --cpu-steps 2 > gpurun_out/bench_long.json 2> gpurun_out/bench_long.err || { tail -20 gpurun_out/bench_long.err; exit 1; }
cut -c1-300 gpurun_out/bench_long.json
