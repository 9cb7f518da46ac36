#!/bin/bash
# Round-4 final checks on one box: the full GPU suite and smoke (as the driver runs them), the
# driver's bench line, and the tools build's engine tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step gputests 1000 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 150 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python -u bench.py
step tools_tests 600 env GOL_AMD_LIB=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so python -u -m pytest tests/test_gpu_engine.py -m gpu -q --maxfail=5 --timeout 150 --timeout-method thread
