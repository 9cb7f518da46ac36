set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/launch_table.py --size 65536 --mv 8,10 --k 8,16 > gpurun_out/g45_lt.log 2>&1; echo "lt rc=$?"; grep '"mv"' gpurun_out/g45_lt.log
timeout -k 10 300 python -u tools/launch_table.py --size 16384 --mv 8,10 --k 8,16 --reps 20 > gpurun_out/g45_lt16.log 2>&1; echo "lt16 rc=$?"; grep '"mv"' gpurun_out/g45_lt16.log
