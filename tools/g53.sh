set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/launch_table.py --size 65536 --mv 8,10 --k 8,16 --band 607 > gpurun_out/g53_lt.log 2>&1; echo "lt rc=$?"; grep '"mv"' gpurun_out/g53_lt.log
timeout -k 10 300 python -u tools/launch_table.py --size 65536 --mv 8,10 --k 8,16 --band 547 > gpurun_out/g53_lt2.log 2>&1; echo "lt2 rc=$?"; grep '"mv"' gpurun_out/g53_lt2.log
