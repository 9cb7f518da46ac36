#!/bin/bash
# Round-4 probe 13: K1p / K1q on cached block buffers with the release / acquire hand-off:
# parity, the C2 autotune's K1p timing, then the product suite, smoke and the bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
T=$PWD/conway-s-gol-distributed_amd/build/libgolamd_tools.so
step() { local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
step k1p_parity 300 python -u -m pytest tests/test_gpu_engine.py -q --timeout 150 --timeout-method thread -k "tile_persist_pinned or spin_timeout or small_board"
step c2_auto 200 env GOL_AUTOTUNE_LOG=1 python -u tools/tile_sweep.py --size 5120 --auto --turns 960 --rounds 3
step k1q_parity 300 env GOL_AMD_LIB=$T python -u -m pytest tests/test_gpu_engine.py -q --timeout 150 --timeout-method thread -k "tile_stream_pinned"
step gputests 1000 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 150 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python -u bench.py
