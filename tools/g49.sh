set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "workgroup and not digests" > gpurun_out/g49_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/g49_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/launch_table.py --size 65536 --mv 9,12 --k 8,12,16 > gpurun_out/g49_lt.log 2>&1; echo "lt rc=$?"; grep '"mv"' gpurun_out/g49_lt.log
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 0 --tpl 16 --mw 1 --mv 9,12 --turns 960 > gpurun_out/g49_sw16.log 2>&1; echo "sw16 rc=$?"; grep -v amdgpu gpurun_out/g49_sw16.log
timeout -k 10 300 python -u tools/launch_table.py --size 65536 --mv 9 --k 8,16 --band 607 > gpurun_out/g49_lt607.log 2>&1; echo "lt607 rc=$?"; grep '"mv"' gpurun_out/g49_lt607.log
timeout -k 10 300 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 0 --rccl direct > gpurun_out/g49_strip8.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g49_strip8.log
