set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 200 --no-cpu-baseline --c3-size 0 > gpurun_out/g30_b20w200.log 2>&1; rc=$?; echo "b20w200 rc=$rc"; tail -1 gpurun_out/g30_b20w200.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu-baseline --c3-size 0 > gpurun_out/g30_b200.log 2>&1; rc=$?; echo "b200 rc=$rc"; tail -1 gpurun_out/g30_b200.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt20 -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 > $R/gpurun_out/g30_kt20.log 2>&1; echo "kt20 rc=$?"
