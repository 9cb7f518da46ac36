#!/bin/bash
# Round-4 probe 11: 4-wave ORD 5 workgroups at 65536^2 (barrier among 4 waves, 6 per CU), then
# the profile refresh with the headline alternates
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/tile_sweep.py --size 65536 --turns 480 --rounds 3 --shapes 14:720:524:24,14:336:524:24,14:344:524:20,30:536:524:20 > gpurun_out/sweep65_4w.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep65_4w.log
ALT_HEADLINE=30:336:524:20,30:344:524:20,14:720:524:20,30:536:524:20,14:720:524:24,30:336:524:24,14:728:524:20,30:528:524:24 bash tools/profile_r04.sh
