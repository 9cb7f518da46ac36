#!/bin/bash
# Round-4 last check: the autotune's long re-timing at 65536^2 (log), then the suite, smoke
# and the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 65536 --turns 960 --rounds 2 --auto > gpurun_out/auto65_long.log 2>&1 || exit $?
grep "autotune long\|^{" gpurun_out/auto65_long.log
bash tools/r04_final.sh
