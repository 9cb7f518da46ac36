cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 200 python -u tools/strip_emulate.py --n 2,4,8 --halo 20 --rccl direct --turns 640 > gpurun_out/ovl_plain_$r.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/strip_emulate.py --n 2,4,8 --halo 20 --rccl direct --overlap --turns 640 > gpurun_out/ovl_on_$r.log 2>&1 || exit $?
done
