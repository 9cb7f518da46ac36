#!/bin/bash
# Round-4 probe 15 (informational): the tools build's autotune timing K1q (cached hand-off)
# against the tuned steady rate at 65536^2 and 16384^2
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
T=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so
for n in 65536 16384; do
  timeout -k 10 300 env GOL_AMD_LIB=$T GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size $n --turns 960 --rounds 2 --auto > gpurun_out/auto_tools_$n.log 2>&1 || exit $?
  grep "autotune stream\|^{" gpurun_out/auto_tools_$n.log
done
