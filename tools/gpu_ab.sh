cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/kbench.py --opt 0=0,1 > gpurun_out/kbench_stagger.log 2>&1 || { tail -20 gpurun_out/kbench_stagger.log; exit 1; }
cat gpurun_out/kbench_stagger.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2>gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
