# exec-masked halo stores in the shipped kernel: parity + timing
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
t() { timeout -k 10 300 "$@" 2>&1 | grep -v amdgpu.ids; }
j() { python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['launch_us'], d['config']['band_rows'], d['config']['temporal_blocking_k'])"; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_engine.py > gpurun_out/t_engine.log 2>&1; rc=$?; tail -1 gpurun_out/t_engine.log; [ $rc -ne 0 ] && exit $rc
t python -u tools/occupancy_probe.py --waves 4 --band 256
for i in 1 2; do t python -u bench.py --no-cpu-baseline | j; done
