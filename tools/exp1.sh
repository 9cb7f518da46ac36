# full GPU suite, smoke, then the round-1 profiles of the shipped default
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/t_all.log 2>&1; rc=$?; tail -2 gpurun_out/t_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
rm -rf gpurun_out/prof gpurun_out/pmc_sq_k8il
bash tools/profile.sh || exit 1
TAG=_k8il bash tools/pmc_sq.sh || exit 1
python tools/pmc_report.py gpurun_out/pmc_sq_k8il/run_counter_collection.csv > gpurun_out/pmc_sq_k8il/report.txt
grep -v amdgpu.ids gpurun_out/prof/kt.log | tail -1
