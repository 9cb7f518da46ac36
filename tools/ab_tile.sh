#!/bin/bash
# A/B of k_step_tile builds on one box: every library in $LIBS times the same shapes
# (tools/tile_sweep.py).  usage: LIBS="old new exp2" bash tools/ab_tile.sh SIZE TURNS SHAPES
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
size=$1 turns=$2 shapes=$3
for l in ${LIBS:-old new}; do
  if [ "$l" = new ]; then lib=$PWD/conway-s-gol-distributed_amd/build/libgolamd.so
  else lib=$PWD/conway-s-gol-distributed_amd/build/libgolamd_$l.so; fi
  echo "== $l $size"
  GOL_AMD_LIB=$lib timeout -k 10 200 python -u tools/tile_sweep.py --size "$size" --turns "$turns" \
    --rounds 2 --shapes "$shapes" 2>&1 | grep shape || exit 1
done
