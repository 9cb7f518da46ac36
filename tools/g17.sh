set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g17_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/g17_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -k "temporal or workgroup or large_board or random_vs or strips" > gpurun_out/g17_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/g17_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 0 --rccl direct > gpurun_out/g17_strip8.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g17_strip8.log
timeout -k 10 300 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 0 --rccl direct --overlap > gpurun_out/g17_strip8ov.log 2>&1; echo "stripov rc=$?"; grep '"n"' gpurun_out/g17_strip8ov.log
