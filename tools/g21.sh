set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for P in 0 36000 48000; do
GOL_WG_LDS_PAD=$P timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 27,34,40,45,54 --tpl 12,16 --mw 1 --mv 9 --turns 960 > gpurun_out/g21_sw16_p$P.log 2>&1 || exit 1; echo "sw16 pad=$P"; grep -v amdgpu gpurun_out/g21_sw16_p$P.log
done
