#!/bin/bash
# rocprofv3 passes over the bench (N=1): kernel trace + stats, then one PMC pass per
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/prof"
mkdir -p "$O"
STEPS=${STEPS:-200}
# the kernel-trace pass profiles exactly the driver's default bench command
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o run --output-format csv -- \
  python3 "$R/bench.py" > "$O/kt.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 200 --warmup 8 --no-cpu-baseline > "$O/fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 200 --warmup 8 --no-cpu-baseline > "$O/write.log" 2>&1
rc=$?; echo "write rc=$rc"; exit $rc
