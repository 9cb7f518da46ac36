#!/bin/bash
# Round-4 probe 14: K1q (tools build, cached hand-off) at deeper blocks, beside plain launches
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
T=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; grep '^{' "gpurun_out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step plain 300 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 14:713:524:24,30:528:524:24,14:1064:524:32,30:536:524:20
step q24 300 env GOL_AMD_LIB=$T GOL_STREAM=24 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 14:713:524:24,30:528:524:24
step q32 300 env GOL_AMD_LIB=$T GOL_STREAM=32 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 14:1064:524:32
step q20 300 env GOL_AMD_LIB=$T GOL_STREAM=20 python -u tools/tile_sweep.py --size 65536 --turns 960 --rounds 3 --shapes 30:536:524:20
