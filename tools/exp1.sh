# full GPU suite + smoke + default bench (with CPU baseline)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/t_all.log 2>&1; rc=$?; tail -3 gpurun_out/t_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_full.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/bench_full.log | tail -1; exit $rc
