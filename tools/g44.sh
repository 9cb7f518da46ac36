#!/bin/bash
# PMC FETCH_SIZE / WRITE_SIZE passes (each its own run) for the kernels the final bench line
# names: 65536^2 k_step_skew K = 8 (the 1000-turn run's dominant launch) and 16384^2
# k_step_wg parallelogram K = 16 (configs[2]).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/prof44"
mkdir -p "$O"
run() {  # name seconds args...
  local name=$1 t=$2; shift 2
  timeout -s KILL "$t" rocprofv3 "$@" > "$O/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0
}
run fetch8 180 --pmc FETCH_SIZE -d "$O/fetch8" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 200 --warmup 16 --no-cpu-baseline --c3-size 0 --tpl 8
run write8 180 --pmc WRITE_SIZE -d "$O/write8" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 200 --warmup 16 --no-cpu-baseline --c3-size 0 --tpl 8
run fetch16 180 --pmc FETCH_SIZE -d "$O/fetch16" -o run --output-format csv -- \
  python3 "$R/bench.py" --size 16384 --steps 2400 --warmup 128 --no-cpu-baseline --c3-size 0
run write16 180 --pmc WRITE_SIZE -d "$O/write16" -o run --output-format csv -- \
  python3 "$R/bench.py" --size 16384 --steps 2400 --warmup 128 --no-cpu-baseline --c3-size 0
echo "g44 done"
