#!/bin/bash
# Round-4 probe 4: K1p at C2 with sibling codes (autotune log); SQ counter passes of the ORD 5
# 65536^2 shapes (30 x 536 K 20, 14 x 720 K 24) and the ORD 1 30 x 576 K 32 for comparison.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step ord6_parity 200 python -u -m pytest tests/test_gpu_engine.py -q --timeout 150 --timeout-method thread -k "tile_code_pinned and (612 or 616 or 624)"
step sweep65f 400 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 30:536:524:20,30:536:624:20,14:720:624:24,14:720:524:24,30:336:624:24,30:336:524:24,30:472:616:20,14:984:616:20
step c2_auto 200 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 5120 --auto --turns 960 --rounds 3
step pmc_o5 300 env TAG=_o5 bash tools/pmc_sq.sh tools/kernel_run.py --size 65536 --mv 15 --tpl 20 --band 536 --tile 30,524 --turns 100
step pmc_o5n 300 env TAG=_o5n bash tools/pmc_sq.sh tools/kernel_run.py --size 65536 --mv 15 --tpl 24 --band 720 --tile 14,524 --turns 96
step pmc_o1 300 env TAG=_o1 bash tools/pmc_sq.sh tools/kernel_run.py --size 65536 --mv 15 --tpl 32 --band 576 --tile 30,140 --turns 96
step clock 200 python -u tools/clock_probe.py
for t in _o5 _o5n _o1; do for p in p1 p2; do
  f=$(ls gpurun_out/pmc_sq$t/$p/*counter_collection.csv gpurun_out/pmc_sq$t/$p/*/*/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 tools/pmc_report.py "$f" > gpurun_out/pmc_sq$t/${p}_report.txt
done; done
echo done
