set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
(go version || echo "go: absent"; nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))") > gpurun_out/g1_env.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/g1_b20.log 2>&1 && \
timeout -k 10 300 python -u bench.py --size 16384 --steps 10000 --warmup 100 --no-cpu-baseline > gpurun_out/g1_b16k.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline > gpurun_out/g1_b1000.log 2>&1
echo done rc=$?
