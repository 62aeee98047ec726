# round 5 / 34: kernel-trace stats of bench.py N=1 on the final tree (bf16 and fp8 flagship)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_34
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp
for dt in bfloat16 float8_e4m3fn; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$dt -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --dtype $dt > $R/$O/bench_$dt.json 2> $R/$O/bench_$dt.err || { tail -20 $R/$O/bench_$dt.err; exit 1; }
  f=$(find /tmp/kt_$dt -name '*kernel_stats.csv' | head -1)
  cp "$f" $R/$O/kernel_stats_$dt.csv
  head -6 $R/$O/kernel_stats_$dt.csv | cut -c1-220
  cut -c1-200 $R/$O/bench_$dt.json
done
