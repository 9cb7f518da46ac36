# per-step overhead ablations of the K=8 IL kernel (wrong results; timing only)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
t() { timeout -k 10 300 "$@" 2>&1 | grep -v amdgpu.ids; }
for v in 6 101 102 103 104 107 6; do echo "== variant $v"; GOL_MULTI_VARIANT=$v t python -u tools/occupancy_probe.py --waves 4 --band 256; done
