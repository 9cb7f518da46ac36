set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for args in "--n 1 --offset 0 --check" "--n 2 --offset 0" "--n 2 --offset 8 --check" "--n 4 --offset 4" "--n 4 --offset 8 --check" "--n 3 --offset 5"; do
timeout -k 10 200 python -u tools/substrip_proto.py --size 16384 --windows 8 $args > gpurun_out/g43.log 2>&1; rc=$?; echo "rc=$rc $args"; grep '"size"' gpurun_out/g43.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/g43.log; exit $rc; }
done
