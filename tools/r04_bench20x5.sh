#!/bin/bash
# The driver's 20-turn headline in 5 fresh processes (plan choice and clock spread)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --c3-size 0 --c2-size 0 --no-c1 > gpurun_out/b20_$i.log 2>&1 || exit $?
  grep '^{"metric' gpurun_out/b20_$i.log | cut -c1-160
done
