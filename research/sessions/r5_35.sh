# round 5 / 35: per-launch duration sequence of the flagship pt4 (kernel trace), to see what the
# 97-136 us spread of r5_34 is made of (warm-up, periodic, random)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_35
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o kt -- python3 $R/scripts/bench_gemm.py --shapes 0 --tiles auto --rounds 10 --iters 40 > $R/$O/bench.txt 2>&1 || { tail $R/$O/bench.txt; exit 1; }
f=$(find /tmp/kt -name '*kernel_trace.csv' | head -1)
python3 - "$f" > $R/$O/durations.txt <<'PY'
import csv, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "pt4" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows]
st = [int(r["Start_Timestamp"]) for r in rows]
gaps = [(st[i + 1] - int(rows[i]["End_Timestamp"])) / 1000 for i in range(len(rows) - 1)]
print("launches", len(d), "median", statistics.median(d), "min", min(d), "max", max(d))
for i in range(0, len(d), 40):
    blk = d[i:i + 40]
    print(f"block {i // 40}: first5 {[round(x, 1) for x in blk[:5]]} median {statistics.median(blk):.1f} min {min(blk):.1f}")
even, odd = d[0::2], d[1::2]
print("even/odd medians", statistics.median(even), statistics.median(odd))
print("gap median us", statistics.median(gaps) if gaps else None)
PY
cat $R/$O/durations.txt
