# kernel-to-kernel gaps in the N=8 strip loop (rocprofv3 kernel trace)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/gap -o run --output-format csv -- python3 $R/tools/strip_emulate.py --n 8 --halo 128 --tpl 0 --band 0 --turns 1024 > $R/gpurun_out/gap.log 2>&1 || exit 1
cd $R
python - <<'PY'
import csv, glob, statistics
f = glob.glob("gpurun_out/gap/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-200:]
gaps, durs = [], []
for a, b in zip(rows, rows[1:]):
    gaps.append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
for r in rows:
    durs.append(((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Kernel_Name"][:50]))
import collections
c = collections.Counter(n for _, n in durs)
print(c.most_common(6))
print("gap us median", statistics.median(gaps), "mean", statistics.mean(gaps), "max", max(gaps))
sk = [d for d, n in durs if "skew" in n]
print("skew dur us median", statistics.median(sk), "n", len(sk))
PY
grep -v amdgpu.ids gpurun_out/gap.log | tail -2
