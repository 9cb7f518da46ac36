set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/sweep.py --size 65536 --variants 2 --bands 0 --tpl 8,16 --mw 1 --mv 8,9,10 --turns 240 > gpurun_out/g5_sw65.log 2>&1; echo "sw65 rc=$?"; grep -v amdgpu gpurun_out/g5_sw65.log
