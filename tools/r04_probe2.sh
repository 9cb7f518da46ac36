#!/bin/bash
# Round-4 probe 2: K1p debug variants, ORD 5 parity, 65536^2 / 16384^2 shapes at 6 and 5
# waves per SIMD (ORD 5), C2 autotune with K1p.  rc 1 = a failed check: the next step runs;
# anything else ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step persist_debug 200 python -u tools/persist_debug.py
step ord5_parity 400 python -u -m pytest tests/test_gpu_engine.py -q --timeout 150 --timeout-method thread -k "tile_persist_pinned or (tile_code_pinned and (503 or 504 or 506 or 508 or 512 or 516 or 524 or 532 or 540))"
step sweep65d 400 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 30:472:116:20,30:536:524:20,14:1112:524:20,30:600:532:20,30:600:540:20,30:600:140:20,62:248:524:20,30:536:424:20,30:504:524:32,30:576:532:32,30:576:140:32
step sweep16d 300 python -u tools/tile_sweep.py --size 16384 --turns 640 --rounds 3 --auto --shapes 14:320:106:32,14:320:506:32,14:320:406:32,30:576:524:32,14:1088:524:32,30:448:516:32
step c2_auto 200 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 5120 --auto --turns 960 --rounds 3
