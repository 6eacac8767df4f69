#!/bin/bash
# r04 batch m: SQ counters of the b0.c2 forward (kbench layer 3) on the K-tile-image kernel vs the W-halo kernel
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmcm_$v -o run -- python3 tools/kbench.py --iters 3 --only fwd --layer 3 --set 18=$v > gpurun_out/pmcm_$v.log 2>&1 || { tail -5 gpurun_out/pmcm_$v.log; exit 1; }
  echo "== option 18 = $v"; grep -E "fwd" gpurun_out/pmcm_$v.log | tail -1
  python3 tools/pmc_sq_summary.py gpurun_out/pmcm_$v gemm
done
