#!/bin/bash
# Round-4 probe 12: K1q (tools build) with cached block buffers and agent release / acquire
# fences; then the product GPU suite again (the product library was rebuilt)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
T=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step k1q_parity 300 env GOL_AMD_LIB=$T python -u -m pytest tests/test_gpu_engine.py -q --timeout 150 --timeout-method thread -k "tile_stream_pinned"
step k1q_sweep 300 env GOL_AMD_LIB=$T GOL_STREAM=20 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 30:536:524:20
step k1q_debug 300 env GOL_AMD_LIB=$T python -u tools/k1q_debug.py
step gputests 1000 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 150 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
