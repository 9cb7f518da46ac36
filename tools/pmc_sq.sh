#!/bin/bash
# SQ / GRBM counter pass over a short bench run (one rocprofv3 pass, <= 8 SQ + 2 GRBM).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/pmc_sq${TAG:-}"
mkdir -p "$O"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
  SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
  -d "$O" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 6 --no-cpu-baseline ${BENCH_ARGS:-} \
  > "$O/log" 2>&1
echo "pmc_sq rc=$?"
