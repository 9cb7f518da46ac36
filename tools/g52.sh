set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/gpurun_out/ht52 -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 > $R/gpurun_out/g52.log 2>&1; echo "ht rc=$?"; tail -1 $R/gpurun_out/g52.log | cut -c1-120
ls $R/gpurun_out/ht52
