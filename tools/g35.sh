set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
T=${TAG:-g35}
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "workgroup and not digests and (12 or 16)" > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 43,55,67 --tpl 16 --mw 1 --mv 12 --turns 960 > gpurun_out/${T}_sw16.log 2>&1 || exit 1; echo "sw16"; grep -v amdgpu gpurun_out/${T}_sw16.log
timeout -k 10 300 python -u tools/sweep.py --size 65536 --variants 2 --bands 607 --tpl 16 --mw 1 --mv 9,12 --turns 480 > gpurun_out/${T}_sw65.log 2>&1 || exit 1; echo "sw65"; grep -v amdgpu gpurun_out/${T}_sw65.log
timeout -k 10 300 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 0 --rccl direct > gpurun_out/${T}_strip8.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/${T}_strip8.log
