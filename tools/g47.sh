set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for p in 3210 3102 3012 2103 3213 3003 2112 0000; do
GOL_WG_PRIO=$p timeout -k 10 200 python -u tools/launch_table.py --size 65536 --mv 9 --k 8,16 --band 607 > gpurun_out/g47.log 2>&1 || exit 1; echo "prio $p"; grep '"mv"' gpurun_out/g47.log
GOL_WG_PRIO=$p timeout -k 10 200 python -u tools/launch_table.py --size 16384 --mv 12 --k 16 --band 55 --reps 20 > gpurun_out/g47b.log 2>&1 || exit 1; grep '"mv"' gpurun_out/g47b.log
done
