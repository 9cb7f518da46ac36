# round-1 profiles of the shipped default: kernel trace + stats, FETCH/WRITE, SQ counters
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/profile.sh || exit 1
TAG=_k8il bash tools/pmc_sq.sh || exit 1
python tools/pmc_report.py gpurun_out/pmc_sq_k8il/run_counter_collection.csv > gpurun_out/pmc_sq_k8il/report.txt
cat gpurun_out/pmc_sq_k8il/report.txt
tail -1 gpurun_out/prof/kt.log
