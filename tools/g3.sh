set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -k "workgroup or temporal_blocking_strips" > gpurun_out/g3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g3_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/sweep.py --size 65536 --variants 2 --bands 0 --tpl 8,12,16 --mw 1 --mv 8 --turns 240 > gpurun_out/g3_sw65_wg.log 2>&1; echo "sw65 rc=$?"; cat gpurun_out/g3_sw65_wg.log | grep -v amdgpu
timeout -k 10 300 python -u tools/sweep.py --size 65536 --variants 2 --bands 0 --tpl 8 --mw 1 --mv 7 --turns 240 > gpurun_out/g3_sw65_skew.log 2>&1; echo "sw65s rc=$?"; cat gpurun_out/g3_sw65_skew.log | grep -v amdgpu
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 0 --tpl 8,12,16 --mw 1 --mv 8 --turns 960 > gpurun_out/g3_sw16_wg.log 2>&1; echo "sw16 rc=$?"; cat gpurun_out/g3_sw16_wg.log | grep -v amdgpu
timeout -k 10 300 env GOL_MULTI_VARIANT=8 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 0,8,12,16 --rccl direct > gpurun_out/g3_strip8_wg.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g3_strip8_wg.log
