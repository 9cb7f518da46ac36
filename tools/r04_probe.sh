#!/bin/bash
# Round-4 probes on one GPU box (each step has its own limit; a failing step ends the script).
#   PART=tests : the round's new GPU tests + the C2 (5120^2) autotune with and without K1p
#   PART=perf  : the stencil mix's issue rate at every occupancy; 65536^2 tile shapes at
#                K = 20 with the barrier (ORD 1) and with neighbour flags (ORD 4); SQ
#                counter passes of the two main shapes (PMC=1)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
# (rc 1 = test failures or a failed check: reported, the next step still runs; anything
# else -- a crash, abort, fault or time limit -- ends the script)
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
B=conway-s-gol-distributed_amd/build
if [ "${PART:-all}" != perf ]; then
  step new_tests 700 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_run.py -v --timeout 150 --timeout-method thread -k "tile_code or tile_persist or spin_timeout or driver_command or stub_harness or keys_mid_run or small_board or planner or event_sequence or keys_save or multi_strip or 5120"
  step c2_auto 200 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 5120 --auto --turns 960 --rounds 3
  step c2_nopersist 200 env GOL_NO_PERSIST=1 python -u tools/tile_sweep.py --size 5120 --auto --turns 960 --rounds 3
fi
if [ "${PART:-all}" != tests ]; then
  step calib_occ 120 tools/calib/valu_issue 20000 occupancy
  SHAPES=${SHAPES:-14:984:116:20,14:984:416:20,30:472:116:20,30:472:416:20,30:600:140:20,30:600:440:20,30:536:124:20,30:536:424:20,30:1240:140:20,30:1240:440:20,62:600:140:20,62:600:440:20}
  step sweep65c 400 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes "$SHAPES"
  if [ -n "${PMC:-}" ]; then
    step pmc_s16 200 env TAG=_s16 bash tools/pmc_sq.sh tools/kernel_run.py --size 65536 --mv 15 --tpl 20 --band 984 --tile 14,416 --turns 100
    step pmc_s40 200 env TAG=_s40 bash tools/pmc_sq.sh tools/kernel_run.py --size 65536 --mv 15 --tpl 20 --band 600 --tile 30,140 --turns 100
  fi
fi
