cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
t() { timeout -k 10 200 "$@" 2>&1 | grep -v amdgpu.ids; }
echo "== bench default"; t python -u bench.py --steps 400 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['launch_us'], d['config']['band_rows'])"
echo "== bench mv3"; GOL_MULTI_VARIANT=3 t python -u bench.py --steps 400 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['launch_us'], d['config']['band_rows'])"
echo "== bench mv3 band137 tpl8"; GOL_MULTI_VARIANT=3 t python -u bench.py --steps 400 --band 137 --tpl 8 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['launch_us'], d['config']['band_rows'])"
echo "== sweep single"; t python -u tools/sweep.py --variants 2 --bands 137 --tpl 8 --mw 1 --mv 1,3 --turns 400 --rounds 5
