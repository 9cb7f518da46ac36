#!/bin/bash
# Round-4 probe 10: where K1q's per-turn time goes -- SQ counter passes of k_tile_stream and of
# plain k_step_tile launches on the same 30 x 536 tiles (65536^2, K = 20, 480 turns)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step pmc_q 300 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so TAG=_q bash tools/pmc_sq.sh tools/kernel_run.py --size 65536 --mv 15 --tpl 20 --band 536 --tile 30,524 --stream 20 --turns 480
step pmc_t 300 env TAG=_t bash tools/pmc_sq.sh tools/kernel_run.py --size 65536 --mv 15 --tpl 20 --band 536 --tile 30,524 --turns 480
step k1q_debug 300 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u tools/k1q_debug.py
for t in _q _t; do for p in p1 p2; do
  f=$(ls gpurun_out/pmc_sq$t/$p/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 tools/pmc_report.py "$f" > gpurun_out/pmc_sq$t/${p}_report.txt
done; done
echo done
