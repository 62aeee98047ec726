# round 5 / 32: kernel-trace durations, back-to-back launches (bench_gemm, 5 rounds x 20 iters), of
# the flagship and 65536x1024x8192 pt4: DEFER vs ONE
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_32
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp
for v in defer one; do
  if [ $v = one ]; then export DDLB_PT4_ONE=1; else unset DDLB_PT4_ONE; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$v -o kt -- python3 $R/scripts/bench_gemm.py --shapes 0,2 --tiles auto --rounds 5 --iters 20 > $R/$O/bench_$v.txt 2>&1 || { tail $R/$O/bench_$v.txt; exit 1; }
  f=$(find /tmp/kt_$v -name '*kernel_stats.csv' | head -1)
  grep -i "pt4" "$f" | cut -d, -f1-8 | cut -c1-60,150-400 > $R/$O/kstats_$v.txt
  cat $R/$O/kstats_$v.txt
  grep "native\|linear" $R/$O/bench_$v.txt
done
