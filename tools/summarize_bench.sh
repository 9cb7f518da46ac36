#!/bin/bash
# Summaries of a tools/profile_bench.sh run (gpurun_out/prof_$ROUND) into
# profiles/${ROUND}_k{K}_{size}_{name}_summary.json:
# the bench's own boards (h = headline, c3, c2: trace of the bench run + pinned PMC passes)
# and the headline alternates (h2.., pinned passes only).
set -eu
R="$(cd "$(dirname "$0")/.." && pwd)"
ROUND=${ROUND:-r06}
O="$R/gpurun_out/prof_$ROUND"
board_of() { case $1 in h) echo 0;; c3) echo 1;; c2) echo 2;; *) echo -;; esac; }
while read -r name size k shape args; do
  kid=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['kernel'])" "$shape")
  case $kid in 15) kn=k_step_tile;; 16) kn=k_tile_persist;; 17) kn=k_tile_stream;; 7) kn=k_step_skew;; *) kn=k_step_wg;; esac
  b=$(board_of "$name")
  kt=kt; [ "$b" = - ] && { kt=-; b=0; }
  python3 "$R/tools/summarize_profile.py" "${ROUND}_k${k}_${size}_${name}" "$O" "$kt" \
    "fetch_$name" "write_$name" "$b" "$kn" "$shape" "sq_$name" "ktpin_$name" > /dev/null
  echo "${ROUND}_k${k}_${size}_${name}"
done < "$O/${PINS:-pins.txt}"
