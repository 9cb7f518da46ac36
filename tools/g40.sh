set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/g40_b20_$i.log 2>&1; rc=$?; echo "b20 rc=$rc"; tail -1 gpurun_out/g40_b20_$i.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
done
