# early stage-0 LDS read (mv8) vs IL (mv6)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
t() { timeout -k 10 300 "$@" 2>&1 | grep -v amdgpu.ids; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_engine.py -k "variants" > gpurun_out/t_var.log 2>&1; rc=$?; tail -2 gpurun_out/t_var.log; [ $rc -ne 0 ] && exit $rc
echo "== sweep8"; t python -u tools/sweep.py --variants 2 --bands 137,274 --tpl 8 --mw 1 --mv 6,8 --turns 400 --rounds 3
echo "== sweep6"; t python -u tools/sweep.py --variants 2 --bands 137,274 --tpl 6 --mw 1 --mv 6,8 --turns 240 --rounds 3
