#!/bin/bash
# N-rank (N=${N:-2}) data-parallel rehearsal on ONE GPU: gloo over GPU tensors, per-step LSTM launches (the
# persistent LSTM kernels need the whole chip and must not run from two processes at once)
cd $GRAFT_REPO_ROOT
export CRNN_SHARE_DEVICE=1 CRNN_DIST_BACKEND=gloo CRNN_LSTM_PER_STEP=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${N:-2} --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus ${N:-2} --steps 3 --warmup 1 --batch ${BATCH:-64} > gpurun_out/dp${N:-2}.json 2> gpurun_out/dp${N:-2}.err || { tail -30 gpurun_out/dp${N:-2}.err; exit 1; }
cat gpurun_out/dp${N:-2}.json | cut -c1-400
