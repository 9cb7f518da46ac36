set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
GOL_AUTOTUNE_LOG=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/g41_b20.log 2>&1; rc=$?; echo "b20 rc=$rc"; tail -1 gpurun_out/g41_b20.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['launch_plan'], d['configs_measured'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 0 --rccl direct > gpurun_out/g41_strip8.log 2>&1; echo "strip rc=$?"; grep '"n"' gpurun_out/g41_strip8.log
