#!/bin/bash
# Round-4 probe 5: staged wave priorities (libgolamd_prio.so) against the product build on the
# 65536^2 ORD 5 shapes; the N = 8 / 4 strip emulation with the ORD 5 family in the search.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
B=conway-s-gol-distributed_amd/build
S65=14:720:524:24,30:536:524:20,30:336:524:24,14:528:524:24,14:720:524:20,30:344:524:20
step prio_parity 200 env GOL_AMD_LIB=$PWD/$B/libgolamd_prio.so python -u -m pytest tests/test_gpu_engine.py -q --timeout 150 --timeout-method thread -k "tile_code_pinned and (516 or 524 or 624 or 406)"
step sweep65_base 300 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes $S65
step sweep65_prio 300 env GOL_AMD_LIB=$PWD/$B/libgolamd_prio.so python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes $S65
step strips 500 env GOL_AUTOTUNE_LOG=1 python -u tools/strip_emulate.py --n 8,4 --halo 128 --rccl direct --turns 768
