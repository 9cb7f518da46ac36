set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 60 --timeout-method thread -k "workgroup and (tpl8 or -8- or 16-)" > gpurun_out/g10_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/g10_tests.log
timeout -k 10 500 python -u tools/sweep.py --size 65536 --variants 2 --bands 0 --tpl 8,12,16 --mw 1 --mv 8,13,14 --turns 240 > gpurun_out/g10_sw65.log 2>&1; echo "sw65 rc=$?"; grep -v amdgpu gpurun_out/g10_sw65.log
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 0 --tpl 12,16 --mw 1 --mv 13,14 --turns 960 > gpurun_out/g10_sw16.log 2>&1; echo "sw16 rc=$?"; grep -v amdgpu gpurun_out/g10_sw16.log
