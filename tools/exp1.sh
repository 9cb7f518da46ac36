# run driver (pinned PGM I/O) + distributed tests
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_run.py > gpurun_out/t_run.log 2>&1; rc=$?; tail -2 gpurun_out/t_run.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_distributed.py > gpurun_out/t_dist.log 2>&1; rc=$?; tail -2 gpurun_out/t_dist.log; exit $rc
