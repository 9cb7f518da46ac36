#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/calib"
mkdir -p "$O"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o run --output-format csv -- "$R/tools/calib/calib_fetch" > "$O/fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o run --output-format csv -- "$R/tools/calib/calib_fetch" > "$O/write.log" 2>&1
