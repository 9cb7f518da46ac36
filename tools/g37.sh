set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt37 -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 > $R/gpurun_out/g37_kt20.log 2>&1; echo "kt20 rc=$?"; tail -1 $R/gpurun_out/g37_kt20.log | cut -c1-300
cd $R
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 45 --no-cpu-baseline --c3-size 0 > gpurun_out/g37_w45.log 2>&1; echo "w45 rc=$?"; tail -1 gpurun_out/g37_w45.log | cut -c1-300
