# C2 / C3 end to end through gol.Run
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_run.py -k baseline_configs > gpurun_out/t_c2c3.log 2>&1; rc=$?; tail -5 gpurun_out/t_c2c3.log; exit $rc
