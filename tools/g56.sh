set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for H in 16384 16360 16335 16390; do
timeout -k 10 200 python -u tools/sweep.py --size 16384 --height $H --variants 2 --bands 55 --tpl 16 --mw 1 --mv 12 --turns 960 --rounds 5 > gpurun_out/g56.log 2>&1 || exit 1; echo "H=$H"; grep '"variant"' gpurun_out/g56.log
done
