set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g57_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/g57_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g57_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/g57_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/g57_b20.log 2>&1; rc=$?; echo "b20 rc=$rc"; tail -1 gpurun_out/g57_b20.log | cut -c1-150
