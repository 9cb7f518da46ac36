set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 54,64,68 --tpl 8,12,16 --mw 1 --mv 9 --turns 960 > gpurun_out/g20_sw16.log 2>&1 || exit 1; echo "sw16"; grep -v amdgpu gpurun_out/g20_sw16.log
timeout -k 10 200 python -u tools/wg_diag.py --size 16384 --bands 64,32 --tpl 16,12 > gpurun_out/g20_diag.log 2>&1 || exit 1; echo diag; grep -v amdgpu gpurun_out/g20_diag.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/g20_b20.log 2>&1 || exit 1; echo b20; tail -1 gpurun_out/g20_b20.log
