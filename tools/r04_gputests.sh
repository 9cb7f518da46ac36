#!/bin/bash
# Round-4 full GPU test suite + smoke, as the driver runs them at round end.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 150 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gputests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; exit $rc
