#!/bin/bash
# r04 batch s: HBM bytes per conv forward launch, K-tile-image kernel (option 18 = 0) vs W-halo kernel (1),
# kbench layers 3 (b0.c2, 8x64) and 6 (b3.c2, 4x32); FETCH_SIZE and WRITE_SIZE in separate passes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1; do
  for C in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/pmcs_${v}_${C:0:1}
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $d -o run -- python3 tools/kbench.py --iters 2 --only fwd --set 18=$v > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  done
  echo "== option 18 = $v"
  python3 tools/pmc_kbench_summary.py gpurun_out/pmcs_${v}_F gpurun_out/pmcs_${v}_W | tail -14
done
