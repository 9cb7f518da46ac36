set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/clock_drift.py --calls 45 > gpurun_out/g38_drift.log 2>&1; echo "drift rc=$?"; grep -v amdgpu gpurun_out/g38_drift.log
timeout -k 10 300 python -u tools/clock_drift.py --calls 20 --idle-ms 200 > gpurun_out/g38_drift_idle.log 2>&1; echo "drift_idle rc=$?"; grep -v amdgpu gpurun_out/g38_drift_idle.log
