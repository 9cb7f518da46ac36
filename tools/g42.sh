#!/bin/bash
# Round-2 final pass: smoke, all GPU tests, the driver's bench command, the default bench,
# the 8-strip emulation and a rocprofv3 kernel-trace/stats summary of the driver's command.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g42_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/g42_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/g42_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/g42_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/g42_b20.log 2>&1; rc=$?; echo "b20 rc=$rc"; tail -1 gpurun_out/g42_b20.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/g42_b1000.log 2>&1; rc=$?; echo "b1000 rc=$rc"; tail -1 gpurun_out/g42_b1000.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/strip_emulate.py --n 2,4,8 --halo 128 --tpl 0 --rccl direct > gpurun_out/g42_strips.log 2>&1; echo "strips rc=$?"; grep '"n"' gpurun_out/g42_strips.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt42 -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/g42_kt20.log 2>&1; echo "kt20 rc=$?"
