set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread -k "bench" > gpurun_out/g55_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/g55_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/g55_b20_$i.log 2>&1; rc=$?; echo "b20 rc=$rc"; tail -1 gpurun_out/g55_b20_$i.log | cut -c1-140; [ $rc -eq 0 ] || exit $rc; done
