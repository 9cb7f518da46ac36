# rows in flight: PD 8 vs 14 vs 17
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
t() { timeout -k 10 300 "$@" 2>&1 | grep -v amdgpu.ids; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_engine.py -k "variants" > gpurun_out/t_var.log 2>&1; rc=$?; tail -1 gpurun_out/t_var.log; [ $rc -ne 0 ] && exit $rc
for v in 6 7 8 6 7 8; do echo "== variant $v"; GOL_MULTI_VARIANT=$v t python -u tools/occupancy_probe.py --waves 4 --band 256; done
