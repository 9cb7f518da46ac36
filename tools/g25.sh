set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for D in 0 1 2 3 7 8; do
GOL_PG_DEBUG=$D timeout -k 10 120 python -u tools/sweep.py --size 16384 --variants 2 --bands 68 --tpl 16 --mw 1 --mv 12 --turns 960 > gpurun_out/g25_d$D.log 2>&1 || exit 1; echo "debug=$D"; grep -v amdgpu gpurun_out/g25_d$D.log | grep GCUPS
done
