set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/launch_table.py --size 65536 --mv 7,9,12 --k 4,5,6,7,8,10,12,16,20,24,32 > gpurun_out/g31_lt65.log 2>&1; echo "lt65 rc=$?"; grep '"mv"' gpurun_out/g31_lt65.log
