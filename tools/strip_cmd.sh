# full GPU suite + strip emulation over direct RCCL + default bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/strip
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/strip/t_all.log 2>&1 &&
timeout -k 10 200 python3 -u tools/strip_emulate.py --rccl direct --full --n 2,4,8 --halo 128 > gpurun_out/strip/rccl_direct2.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py > gpurun_out/strip/bench.log 2>&1
