#!/bin/bash
# Round-3 rocprofv3 passes (each its own run; PMC passes never combine with tracing):
#   kt20    kernel trace + stats of the driver's bench command (bench.py --steps 20 --warmup 5):
#           the 65536^2 headline, then configs_measured: 16384^2 x 10000 (C3), 5120^2 x 1000
#           (C2), 512^2 x 100 (C1)
#   fetch5 / write5    FETCH_SIZE / WRITE_SIZE of the 5120^2 board alone (C2's launches)
#   fetch16 / write16  the same for the 16384^2 board (C3)
# then tools/summarize_profile.py writes profiles/r03_*_summary.json.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/prof3"
mkdir -p "$O"
run() {  # name seconds args...
  local name=$1 t=$2; shift 2
  timeout -s KILL "$t" rocprofv3 "$@" > "$O/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0
}
run kt20 400 --kernel-trace --stats -d "$O/kt20" -o run --output-format csv -- \
  python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5
ONE="--no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1"
run fetch5 180 --pmc FETCH_SIZE -d "$O/fetch5" -o run --output-format csv -- \
  python3 "$R/bench.py" --size 5120 --steps 1000 --warmup 64 $ONE
run write5 180 --pmc WRITE_SIZE -d "$O/write5" -o run --output-format csv -- \
  python3 "$R/bench.py" --size 5120 --steps 1000 --warmup 64 $ONE
run fetch16 180 --pmc FETCH_SIZE -d "$O/fetch16" -o run --output-format csv -- \
  python3 "$R/bench.py" --size 16384 --steps 2400 --warmup 120 $ONE
run write16 180 --pmc WRITE_SIZE -d "$O/write16" -o run --output-format csv -- \
  python3 "$R/bench.py" --size 16384 --steps 2400 --warmup 120 $ONE
echo done
