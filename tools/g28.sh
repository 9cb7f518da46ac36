set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g28_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/g28_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/g28_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g28_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/g28_b20.log 2>&1; rc=$?; echo "b20 rc=$rc"; tail -1 gpurun_out/g28_b20.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/sweep.py --size 65536 --variants 2 --bands 601,607 --tpl 16 --mw 1 --mv 9,12 --turns 480 > gpurun_out/g28_sw65.log 2>&1 || exit 1; echo "sw65"; grep -v amdgpu gpurun_out/g28_sw65.log
timeout -k 10 300 python -u tools/sweep.py --size 65536 --variants 2 --bands 538,544,550 --tpl 12 --mw 1 --mv 9,12 --turns 480 > gpurun_out/g28_sw65b.log 2>&1 || exit 1; echo "sw65b"; grep -v amdgpu gpurun_out/g28_sw65b.log
