set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/calib/wave_place > gpurun_out/g29_place.log 2>&1; echo "place rc=$?"; cat gpurun_out/g29_place.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "deep or (temporal_blocking_strips and (40 or 30))" > gpurun_out/g29_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g29_tests.log
[ $rc -eq 0 ] || exit $rc
GOL_AUTOTUNE_LOG=1 timeout -k 10 300 python -u tools/sweep.py --size 65536 --variants 2 --bands 0 --tpl 16,20,24,32 --mw 1 --mv 9 --turns 480 --rounds 2 > gpurun_out/g29_sw65.log 2>&1 || exit 1; echo "sw65"; grep -v amdgpu gpurun_out/g29_sw65.log | grep -v autotune
GOL_AUTOTUNE_LOG=1 timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 0 --tpl 16,20,24,32 --mw 1 --mv 9,12 --turns 960 > gpurun_out/g29_sw16.log 2>&1 || exit 1; echo "sw16"; grep -v amdgpu gpurun_out/g29_sw16.log | grep -v autotune
GOL_AUTOTUNE_LOG=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/g29_b20.log 2>&1; rc=$?; echo "b20 rc=$rc"; tail -1 gpurun_out/g29_b20.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 0 --rccl direct > gpurun_out/g29_strip8.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g29_strip8.log
