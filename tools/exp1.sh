# bench contract tests (1 GPU; 2 gloo ranks on one GPU)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py -k bench > gpurun_out/t_bench.log 2>&1; rc=$?; tail -4 gpurun_out/t_bench.log; exit $rc
