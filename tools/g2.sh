set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_run.py tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread -k "control_word or 65536_strips or baseline_configs or rccl_self or missing_image or cont_resume or keys_save or bench_contract or torchrun_two or alive_counts or event_sequence" > gpurun_out/g2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/g2_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/g2_b20.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/g2_b20.log
