#!/bin/bash
# Round-4 probe 3: K1p selection at C2 (autotune log), ORD 5 shapes around 30 x 536 at
# 65536^2 (depth, round balance) with the autotuned pick, then the driver's bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step c2_auto 200 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 5120 --auto --turns 960 --rounds 3
step sweep65e 500 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --auto --shapes ${SHAPES:-30:536:524:20,30:504:524:20,30:520:524:20,30:536:524:16,30:544:524:16,30:528:524:24,30:472:516:20,30:536:524:12,30:560:524:8}
step bench 600 python -u bench.py
