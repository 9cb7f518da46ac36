set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g26_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/g26_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 60 --timeout-method thread -k "workgroup and 12" > gpurun_out/g26_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g26_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 55,61,67,73 --tpl 16 --mw 1 --mv 9,12 --turns 960 > gpurun_out/g26_sw16.log 2>&1 || exit 1; echo "sw16"; grep -v amdgpu gpurun_out/g26_sw16.log
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 52,58,64,70 --tpl 12 --mw 1 --mv 9,12 --turns 960 > gpurun_out/g26_sw16b.log 2>&1 || exit 1; echo "sw16b"; grep -v amdgpu gpurun_out/g26_sw16b.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -k "workgroup or strips" > gpurun_out/g26_tests2.log 2>&1
rc=$?; echo "tests2 rc=$rc"; tail -3 gpurun_out/g26_tests2.log
