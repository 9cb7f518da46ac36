#!/bin/bash
# Round-4 probe 6: fine ORD 5 shape sweep at 65536^2; the driver's 20-turn headline in 5 fresh
# processes (plan choice).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step sweep65g 400 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 14:720:524:24,14:712:524:24,14:704:524:24,14:724:524:22,14:716:524:26,14:712:524:28,30:336:524:24,30:344:524:22,30:536:524:20,30:540:524:18
for i in 1 2 3 4 5; do
  step bench20_$i 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1
done
