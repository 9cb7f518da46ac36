set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 60 --timeout-method thread -k "temporal_blocking_interleaved" > gpurun_out/g14_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/g14_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/sweep.py --size 65536 --variants 2 --bands 0 --tpl 8,10,12 --mw 1 --mv 7 --turns 240 > gpurun_out/g14_sw65.log 2>&1; echo "sw65 rc=$?"; grep -v amdgpu gpurun_out/g14_sw65.log
for t in 8 10; do timeout -k 10 300 env GOL_MULTI_VARIANT=7 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --tpl $t > gpurun_out/g14_b20_$t.log 2>&1; echo "b20 tpl$t rc=$?"; tail -1 gpurun_out/g14_b20_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['band_rows'], d['roofline']['launches'], d['roofline']['launch_us'])"; done
timeout -k 10 300 python -u tools/sweep.py --size 16384 --variants 2 --bands 0 --tpl 8,10,12 --mw 1 --mv 7 --turns 960 > gpurun_out/g14_sw16.log 2>&1; echo "sw16 rc=$?"; grep -v amdgpu gpurun_out/g14_sw16.log
