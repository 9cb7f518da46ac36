#!/bin/bash
# Round-4 probe 9: K1q / K1p with cached (hipMalloc) block buffers and write-through sc1 stores
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step stream_parity9 300 python -u -m pytest tests/test_gpu_engine.py -q --timeout 150 --timeout-method thread -k "tile_stream_pinned"
step sweep65_p9 300 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 30:536:524:20,14:713:524:24
step sweep65_s9 300 env GOL_STREAM_LOG=1 GOL_STREAM=20 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 30:536:524:20
step sweep65_s9b 300 env GOL_STREAM_LOG=1 GOL_STREAM=24 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 14:713:524:24
