# interleaved layout as the default: full engine parity, smoke, timing
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
t() { timeout -k 10 300 "$@" 2>&1 | grep -v amdgpu.ids; }
j() { python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['launch_us'], d['config']['band_rows'], d['config']['temporal_blocking_k'])"; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_engine.py > gpurun_out/t_engine.log 2>&1; rc=$?; tail -3 gpurun_out/t_engine.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
echo "== bench default"; t python -u bench.py --no-cpu-baseline | j
echo "== sweep8"; t python -u tools/sweep.py --variants 2 --bands 137,192,240,274,320 --tpl 8 --mw 1 --mv 6 --turns 400 --rounds 3
echo "== sweep6"; t python -u tools/sweep.py --variants 2 --bands 137,192,274 --tpl 6 --mw 1 --mv 6 --turns 240 --rounds 3
