set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 60 --timeout-method thread -k "workgroup or large_board or 65536" > gpurun_out/g13_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/g13_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/g13_b20.log 2>&1; echo "b20 rc=$?"; tail -1 gpurun_out/g13_b20.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config'], d['roofline']['kernel'], d['configs_measured'])"
timeout -k 10 300 python -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline --c3-size 0 > gpurun_out/g13_b1000.log 2>&1; echo "b1000 rc=$?"; tail -1 gpurun_out/g13_b1000.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config'])"
timeout -k 10 300 env GOL_MULTI_VARIANT=8 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 > gpurun_out/g13_b20wg.log 2>&1; echo "b20wg rc=$?"; tail -1 gpurun_out/g13_b20wg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config'])"
timeout -k 10 300 python -u tools/strip_emulate.py --n 2,4,8 --halo 128 --tpl 0 --rccl direct --full > gpurun_out/g13_strips.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g13_strips.log
