#!/bin/bash
# Round-3 (second pass) rocprofv3 passes of the headline board alone, as the driver runs it
# (bench.py --steps 20 --warmup 5, no other configs): kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in passes of their own.  tools/summarize_profile.py turns them into
# profiles/r03b_k{K}_65536_summary.json for the plan's depth K.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/prof3b"
mkdir -p "$O"
ONE="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1"
run() {  # name seconds args...
  local name=$1 t=$2; shift 2
  timeout -s KILL "$t" rocprofv3 "$@" > "$O/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0
}
[ "${ONLY_K20:-0}" = 1 ] || {
run kt 300 --kernel-trace --stats -d "$O/kt" -o run --output-format csv -- python3 "$R/bench.py" $ONE
run fetch 200 --pmc FETCH_SIZE -d "$O/fetch" -o run --output-format csv -- python3 "$R/bench.py" $ONE
run write 200 --pmc WRITE_SIZE -d "$O/write" -o run --output-format csv -- python3 "$R/bench.py" $ONE
}
# the K1t launch the planner picks for 20 turns on some boxes (1 x 20 turns, 14-word tiles of
# SEG 16, 960 rows), pinned, for its PMC bytes per launch
KR="$R/tools/kernel_run.py --size 65536 --mv 15 --tpl 20 --band 960 --tile 14,116 --turns 200"
run fetchk20 200 --pmc FETCH_SIZE -d "$O/fetchk20" -o run --output-format csv -- python3 $KR
run writek20 200 --pmc WRITE_SIZE -d "$O/writek20" -o run --output-format csv -- python3 $KR
echo done
