#!/bin/bash
# Profiles that reproduce the bench line (ROUND=r05 names the pass: gpurun_out/prof_$ROUND,
# then tools/summarize_bench.sh writes profiles/${ROUND}_k{K}_{size}_{name}_summary.json): (1) the bench exactly as the driver runs it
# (bench.py --gpus 1 --steps 20 --warmup 5, all configs) under --kernel-trace --stats; (2) for
# the headline board, C3 and C2, the launch shape the bench reports (config.launch_shape /
# configs_measured[i].launch_shape), pinned in tools/kernel_run.py (no autotune), under a
# FETCH_SIZE pass, a WRITE_SIZE pass, a kernel trace and an SQ / GRBM pass (clock under load,
# VALU counts) of its own -- so the traffic, the clock and the trace average of each summary
# come from the one instantiation the bench timed.
# Since round 5 the BASELINE sizes run pinned shapes (gol_engine.cpp kKnownShapes), so the
# shape profiled here is the shape every bench run times.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
ROUND=${ROUND:-r06}
O="$R/gpurun_out/prof_$ROUND"
mkdir -p "$O"
run() {  # name seconds args...
  local name=$1 t=$2; shift 2
  timeout -s KILL "$t" rocprofv3 "$@" > "$O/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc; return 0
}
# ONLY_EXTRA=1: the EXTRA_PINS shapes alone (no bench trace; a second call of a long pass)
if [ "${ONLY_EXTRA:-0}" = 1 ]; then
  echo '{}' > "$O/bench_line_extra.json"
  BL="$O/bench_line_extra.json"
else
  run kt 400 --kernel-trace --stats -d "$O/kt" -o run --output-format csv -- \
      python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-cold
  grep '^{"metric"' "$O/kt.log" > "$O/bench_line.json" || { echo "no bench line"; exit 1; }
  BL="$O/bench_line.json"
fi
PINS="$O/pins${ONLY_EXTRA:+_x$ONLY_EXTRA}.txt"
# pinned kernel_run arguments per board: "name size turns args..." lines
python3 - "$BL" > "$PINS" <<'PY'
import json, sys
line = json.load(open(sys.argv[1]))
boards = [("h", line["config"]["board"][0], line["config"]["launch_shape"])] if line else []
for i, c in enumerate(line.get("configs_measured", [])[:2]):
    if "launch_shape" in c:
        size = int(c["workload"].split("x")[0])
        boards.append((["c3", "c2"][i], size, c["launch_shape"]))
# alternates for the headline: the 20-turn plan's tile shape is chosen by timing and shapes
# within ~1 % trade places from box to box (profiles/r04_bench20_fresh_processes.jsonl), so
# the shapes it picks are profiled too -- bench.py uses the summary whose shape matches
import os
h = boards[0][2] if boards else None


def tile_shape(k, th, tw, code, rows):
    seg, G = code % 100, 64 // (tw + 2)
    waves = -(-(-(-(th + 2 * k) // seg)) // G)
    return {"kernel": 15, "turns": k, "band_rows": th, "buffer_rows": rows,
            "tile": {"code": code, "width_words": tw, "width_lanes": tw, "height_rows": th,
                     "seg_rows": seg, "turn_order": code // 100 % 10, "words_per_lane": 1,
                     "waves_per_workgroup": waves}}


for i, alt in enumerate(x for x in os.environ.get("ALT_HEADLINE", "").split(",") if x):
    tw, th, code, k = (int(v) for v in alt.split(":"))
    sh = tile_shape(k, th, tw, code, boards[0][1])
    if sh != h:
        boards.append((f"h{i + 2}", boards[0][1], sh))
# row-strip shapes the N > 1 bench times (EXTRA_PINS="name:width:buffer_rows:K:tw:th:code,..."):
# profiled as a torus of the strip's buffer height -- the same launch grid
for x in (x for x in os.environ.get("EXTRA_PINS", "").split(",") if x):
    name, w, rows, k, tw, th, code = x.split(":")
    boards.append((name, int(w), tile_shape(int(k), int(th), int(tw), int(code), int(rows))))
for name, size, sh in boards:
    k = sh["turns"]
    args = (f"--size {size} --height {sh.get('buffer_rows', size)} "
            f"--mv {15 if sh['kernel'] in (15, 16, 17) else sh['kernel']} --band {sh['band_rows']}")
    if sh["kernel"] == 17:
        t = sh["tile"]
        args += f" --tile {t['width_lanes']},{t['code']} --tpl {sh['block_turns']} --stream {sh['block_turns']}"
    elif sh["kernel"] == 16:
        t = sh["tile"]
        args += f" --tile {t['width_lanes']},{t['code']} --tpl {sh['block_turns']} --persist {sh['block_turns']}"
    elif sh["kernel"] == 15:
        t = sh["tile"]
        args += f" --tile {t['width_lanes']},{t['code']} --tpl {k}"
    else:
        args += f" --tpl {k}"
    turns = k * (10 if size >= 65536 else 40)
    if sh.get("kernel") == 16:
        turns = 4 * k
    if sh.get("kernel") == 17:
        turns = k            # (one launch of the bench's size per step)
    print(name, size, k, json.dumps(sh, separators=(",", ":")), args, "--turns", turns)
PY
cat "$PINS"
while read -r name size k shape args; do
  KR="$R/tools/kernel_run.py $args"
  run "fetch_$name" 200 --pmc FETCH_SIZE -d "$O/fetch_$name" -o run --output-format csv -- python3 $KR
  run "write_$name" 200 --pmc WRITE_SIZE -d "$O/write_$name" -o run --output-format csv -- python3 $KR
  run "ktpin_$name" 200 --kernel-trace --stats -d "$O/ktpin_$name" -o run --output-format csv -- python3 $KR
  run "sq_$name" 200 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$O/sq_$name" -o run --output-format csv -- python3 $KR
  echo "$shape" > "$O/shape_$name.json"
done < "$PINS"
echo done
