set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/wg_diag.py --size 65536 --bands 266,625 --tpl 8,16 > gpurun_out/g33_diag.log 2>&1; echo "diag rc=$?"; grep -v amdgpu gpurun_out/g33_diag.log
