set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 37,43,49,55 --tpl 16,8 --mw 1 --mv 12 --turns 960 > gpurun_out/g27_sw16.log 2>&1 || exit 1; echo "sw16"; grep -v amdgpu gpurun_out/g27_sw16.log
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 34,40,46,52 --tpl 12 --mw 1 --mv 12 --turns 960 > gpurun_out/g27_sw16b.log 2>&1 || exit 1; echo "sw16b"; grep -v amdgpu gpurun_out/g27_sw16b.log
timeout -k 10 300 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 0 --rccl direct > gpurun_out/g27_strip8.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g27_strip8.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/g27_b20.log 2>&1; echo "b20 rc=$?"; tail -1 gpurun_out/g27_b20.log
