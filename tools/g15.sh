set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 60 --timeout-method thread -k "workgroup or temporal_blocking_interleaved" > gpurun_out/g15_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/g15_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 16,24,32,40,48,64 --tpl 12 --mw 1 --mv 8 --turns 960 > gpurun_out/g15_sw16.log 2>&1; echo "sw16 rc=$?"; grep -v amdgpu gpurun_out/g15_sw16.log
timeout -k 10 300 env GOL_WG_PERSIST=0 python -u tools/sweep.py --size 16384 --variants 2 --bands 24,32,64 --tpl 12 --mw 1 --mv 8 --turns 960 > gpurun_out/g15_sw16np.log 2>&1; echo "sw16np rc=$?"; grep -v amdgpu gpurun_out/g15_sw16np.log
timeout -k 10 300 env GOL_MULTI_VARIANT=8 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 12 --band 24,32,48,64,96 --rccl direct > gpurun_out/g15_strip8.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g15_strip8.log
timeout -k 10 400 python -u tools/sweep.py --size 65536 --variants 2 --bands 96,137,192,274,365,625 --tpl 12 --mw 1 --mv 8 --turns 240 > gpurun_out/g15_sw65.log 2>&1; echo "sw65 rc=$?"; grep -v amdgpu gpurun_out/g15_sw65.log
