set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/wg_diag.py --size 65536 --bands 625 --tpl 8,16 > gpurun_out/g34_diag.log 2>&1; echo "diag rc=$?"; grep -v amdgpu gpurun_out/g34_diag.log | grep -E "starts|span|wave 0|wave 3"
timeout -k 10 300 python -u tools/wg_diag.py --size 16384 --bands 64 --tpl 16 > gpurun_out/g34_diag16.log 2>&1; echo "diag16 rc=$?"; grep -v amdgpu gpurun_out/g34_diag16.log | grep -E "starts|span|wave"
