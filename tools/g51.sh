set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 > gpurun_out/g51_b20_$i.log 2>&1; rc=$?; tail -1 gpurun_out/g51_b20_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['launch_us'], d['config']['launch_plan'])"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python -u tools/phase_timing.py > gpurun_out/g51_phase.log 2>&1; grep ms gpurun_out/g51_phase.log
