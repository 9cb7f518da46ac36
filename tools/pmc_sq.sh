#!/bin/bash
# SQ / GRBM counter passes (rocprofv3 --pmc, <= 8 SQ + 2 GRBM counters per pass, one pass per
# run) over a short GPU program: by default a short bench run; otherwise the python script and
# arguments given (e.g. tools/kernel_run.py ... for one pinned kernel without the autotune).
#   TAG=_x bash tools/pmc_sq.sh [script.py args...]
# Pass 1: issue / wait breakdown (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES, all
# in quad-cycles, MI355X_MICROARCH.md); pass 2: scalar, LDS and conflict counts.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/pmc_sq${TAG:-}"
mkdir -p "$O"
if [ $# -gt 0 ]; then
  SCRIPT="$R/$1"; shift; ARGS=("$@")
else
  SCRIPT="$R/bench.py"; ARGS=(--steps 60 --warmup 6 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1 ${BENCH_ARGS:-})
fi
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
  SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
  -d "$O/p1" -o run --output-format csv -- python3 "$SCRIPT" "${ARGS[@]}" > "$O/p1.log" 2>&1
rc=$?; echo "pmc_sq pass 1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
  -d "$O/p2" -o run --output-format csv -- python3 "$SCRIPT" "${ARGS[@]}" > "$O/p2.log" 2>&1
rc=$?; echo "pmc_sq pass 2 rc=$rc"; exit $rc
