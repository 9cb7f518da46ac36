#!/bin/bash
# Round-2 rocprofv3 passes (each its own run; PMC passes never combine with tracing):
#   kt20   kernel trace + stats of the driver's bench command (bench.py --steps 20 --warmup 5)
#   kt1000 kernel trace + stats of the steady-state bench (1000 turns)
#   fetch / write  FETCH_SIZE / WRITE_SIZE of the 65536^2 kernel (200 turns, K = 10)
#   fetch16 / write16  the same for the 16384^2 board (k_step_wg)
#   sq     SQ / GRBM counters of the 65536^2 kernel
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/prof2"
mkdir -p "$O"
run() {  # name seconds args...
  local name=$1 t=$2; shift 2
  timeout -s KILL "$t" rocprofv3 "$@" > "$O/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0
}
run kt20 300 --kernel-trace --stats -d "$O/kt20" -o run --output-format csv -- \
  python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5
run kt1000 300 --kernel-trace --stats -d "$O/kt1000" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 1000 --warmup 20 --no-cpu-baseline --c3-size 0
run fetch 180 --pmc FETCH_SIZE -d "$O/fetch" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 200 --warmup 10 --no-cpu-baseline --c3-size 0 --tpl 10
run write 180 --pmc WRITE_SIZE -d "$O/write" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 200 --warmup 10 --no-cpu-baseline --c3-size 0 --tpl 10
run kt16 300 --kernel-trace --stats -d "$O/kt16" -o run --output-format csv -- \
  python3 "$R/bench.py" --size 16384 --steps 10000 --warmup 120 --no-cpu-baseline --c3-size 0
run fetch16 180 --pmc FETCH_SIZE -d "$O/fetch16" -o run --output-format csv -- \
  python3 "$R/bench.py" --size 16384 --steps 2400 --warmup 120 --no-cpu-baseline --c3-size 0
run write16 180 --pmc WRITE_SIZE -d "$O/write16" -o run --output-format csv -- \
  python3 "$R/bench.py" --size 16384 --steps 2400 --warmup 120 --no-cpu-baseline --c3-size 0
run sq 180 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
  -d "$O/sq" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 60 --warmup 10 --no-cpu-baseline --c3-size 0 --tpl 10
echo "profile_r02 done"
