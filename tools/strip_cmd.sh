# one-GPU strip experiments + the distributed GPU tests
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/strip
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 120 --timeout-method thread > gpurun_out/strip/t_dist.log 2>&1 &&
timeout -k 10 200 python3 -u tools/strip_emulate.py --full --n 2,4,8 --halo 128,256 > gpurun_out/strip/zc.log 2>&1
