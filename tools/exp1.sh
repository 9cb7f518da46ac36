# strip emulation: band sweep per N (IL default kernel)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
t() { timeout -k 10 300 "$@" 2>&1 | grep -v amdgpu.ids; }
t python -u tools/strip_emulate.py --n 2 --halo 128 --tpl 8 --band 0,96,137,192,274 --turns 1024
t python -u tools/strip_emulate.py --n 4 --halo 128 --tpl 8 --band 0,40,48,64,70,96,137 --turns 1024
t python -u tools/strip_emulate.py --n 8 --halo 128 --tpl 8 --band 0,18,24,32,36,48,64 --turns 1024
