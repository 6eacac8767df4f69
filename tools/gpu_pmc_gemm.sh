#!/bin/bash
# SQ counters of the plain-GEMM kernels (tools/gemm_square.py) per variant: "LIB:OPT" pairs in $VARIANTS
# (LIB empty = libcrnn_hip.so). Writes gpurun_out/pmcg_<i>/...; summarize with tools/pmc_gemm_summary.py
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CTR="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"
i=0
for v in $VARIANTS; do
  lib=${v%%:*}; opt=${v##*:}
  if [ -n "$lib" ]; then export CRNN_HIP_LIB=$PWD/rcnn-ocr_amd/crnn_hip/$lib; else unset CRNN_HIP_LIB; fi
  timeout -s KILL 90 rocprofv3 --pmc $CTR --output-format csv -d gpurun_out/pmcg_$i -o run -- python3 tools/gemm_square.py $opt > gpurun_out/pmcg_$i.log 2>&1 || { tail -5 gpurun_out/pmcg_$i.log; exit 1; }
  echo "variant $i = $v"; grep "\^3" gpurun_out/pmcg_$i.log
  i=$((i+1))
done
