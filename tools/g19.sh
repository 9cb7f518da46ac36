set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for R in 0 1; do
GOL_WG_ROTATE=$R timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 54,68,64 --tpl 12,16 --mw 1 --mv 8,9 --turns 960 > gpurun_out/g19_sw16_r$R.log 2>&1 || exit 1; echo "sw16 rot=$R"; grep -v amdgpu gpurun_out/g19_sw16_r$R.log
done
for R in 0 1; do
GOL_WG_ROTATE=$R timeout -k 10 300 python -u tools/sweep.py --size 65536 --variants 2 --bands 0 --tpl 12,16 --mw 1 --mv 8,9 --turns 240 > gpurun_out/g19_sw65_r$R.log 2>&1 || exit 1; echo "sw65 rot=$R"; grep -v amdgpu gpurun_out/g19_sw65_r$R.log
done
GOL_WG_ROTATE=1 timeout -k 10 300 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 0 --rccl direct > gpurun_out/g19_strip8.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g19_strip8.log
