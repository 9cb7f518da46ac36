set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/sweep.py --size 65536 --variants 2 --bands 0 --tpl 12,16 --mw 1 --mv 13,15,16 --turns 240 > gpurun_out/g11_sw65.log 2>&1; echo "sw65 rc=$?"; grep -v amdgpu gpurun_out/g11_sw65.log
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 0 --tpl 12,16 --mw 1 --mv 13,15,16 --turns 960 > gpurun_out/g11_sw16.log 2>&1; echo "sw16 rc=$?"; grep -v amdgpu gpurun_out/g11_sw16.log
timeout -k 10 300 env GOL_MULTI_VARIANT=15 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 12,16 --rccl direct > gpurun_out/g11_strip8.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g11_strip8.log
