#!/bin/bash
# Round-4 probe 8: K1q k_tile_stream parity, then its rate against plain K1t launches at
# 65536^2 (and 16384^2), and the autotune's choice.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step stream_parity 300 python -u -m pytest tests/test_gpu_engine.py -q --timeout 150 --timeout-method thread -k "tile_stream_pinned or tile_persist_pinned"
S65=30:335:524:20,14:713:524:24,30:536:524:20,30:344:524:12,14:744:524:12
step sweep65_plain 300 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes $S65
step sweep65_s20 300 env GOL_STREAM=20 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 30:335:524:20,30:536:524:20
step sweep65_s24 300 env GOL_STREAM=24 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 14:713:524:24
step sweep65_s12 300 env GOL_STREAM=12 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 30:344:524:12,14:744:524:12
step sweep16_s 300 env GOL_STREAM=32 python -u tools/tile_sweep.py --size 16384 --turns 640 --rounds 3 --shapes 14:316:106:32
step auto65 400 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --auto
step bench20_a 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1
step bench1000 400 python -u bench.py --no-cpu-baseline --c2-size 0 --no-c1
