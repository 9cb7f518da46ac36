set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -k "workgroup" > gpurun_out/g4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g4_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/sweep.py --size 65536 --variants 2 --bands 0 --tpl 8,12,16 --mw 1 --mv 9,10 --turns 240 > gpurun_out/g4_sw65.log 2>&1; echo "sw65 rc=$?"; grep -v amdgpu gpurun_out/g4_sw65.log
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 0 --tpl 8,12,16 --mw 1 --mv 9 --turns 960 > gpurun_out/g4_sw16.log 2>&1; echo "sw16 rc=$?"; grep -v amdgpu gpurun_out/g4_sw16.log
timeout -k 10 300 env GOL_MULTI_VARIANT=9 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 8,12,16 --rccl direct > gpurun_out/g4_strip8.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g4_strip8.log
