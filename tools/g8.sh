set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/wg_diag.py --bands 274,874 --tpl 8,16 > gpurun_out/g8_diag.log 2>&1; echo "diag rc=$?"; grep -v amdgpu gpurun_out/g8_diag.log
timeout -k 10 300 python -u tools/wg_diag.py --size 16384 --bands 64 --tpl 16 > gpurun_out/g8_diag16.log 2>&1; echo "diag16 rc=$?"; grep -v amdgpu gpurun_out/g8_diag16.log
