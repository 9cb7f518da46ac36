set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -k "planner or control_word or strips_in_process or 65536_strips" > gpurun_out/g36_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/g36_tests.log
[ $rc -eq 0 ] || exit $rc
GOL_AUTOTUNE_LOG=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/g36_b20.log 2>&1; rc=$?; echo "b20 rc=$rc"; grep -E "autotune (plan|launch)" gpurun_out/g36_b20.log | grep -v "^$" | head -80; tail -1 gpurun_out/g36_b20.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --c3-size 0 --no-cpu-baseline > gpurun_out/g36_b20b.log 2>&1; echo "b20b rc=$?"; tail -1 gpurun_out/g36_b20b.log | cut -c1-400
timeout -k 10 300 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 0 --rccl direct > gpurun_out/g36_strip8.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g36_strip8.log
