# round-1 profiles of the shipped default (kernel trace + stats, FETCH/WRITE of the timed launches, SQ)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
rm -rf gpurun_out/prof gpurun_out/pmc_sq_k8il
bash tools/profile.sh || exit 1
TAG=_k8il bash tools/pmc_sq.sh || exit 1
python tools/pmc_report.py gpurun_out/pmc_sq_k8il/run_counter_collection.csv > gpurun_out/pmc_sq_k8il/report.txt
grep -A14 "k_step_skew<8" gpurun_out/pmc_sq_k8il/report.txt | head -16
