#!/bin/bash
# Round-4 probe 7: bench.py's 20-turn measurement repeated in one process; 16384^2 shapes
# with fewer halo rows (ORD 5 / ORD 1 SEG 12 on 704-row tiles).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step bench20_probe 200 python -u tools/bench20_probe.py
step sweep16e 300 python -u tools/tile_sweep.py --size 16384 --turns 640 --rounds 3 --auto --shapes 14:316:106:32,14:704:512:32,14:680:512:32,14:704:112:32,14:320:506:32,30:320:512:32,14:704:612:32,14:456:508:24
# the tools build's kernels under their own tests, once
if [ -f conway-s-gol-distributed_amd/build/libgolamd_tools.so ]; then
  step tools_tests 600 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u -m pytest tests/test_gpu_engine.py -m gpu -q --maxfail=5 --timeout 150 --timeout-method thread
fi
