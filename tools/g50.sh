set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "workgroup and not digests" > gpurun_out/g50_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g50_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/launch_table.py --size 65536 --mv 9,13,12,14 --k 8,12,16 > gpurun_out/g50_lt.log 2>&1; echo "lt rc=$?"; grep '"mv"' gpurun_out/g50_lt.log
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 0 --tpl 16 --mw 1 --mv 12,14,13 --turns 960 > gpurun_out/g50_sw16.log 2>&1; echo "sw16 rc=$?"; grep -v amdgpu gpurun_out/g50_sw16.log
timeout -k 10 300 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 0 --rccl direct > gpurun_out/g50_strip8.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g50_strip8.log
