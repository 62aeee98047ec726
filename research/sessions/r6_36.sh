# round 6 / 36: final-tree (stage_ab + SPLIT) kernel-trace stats of bench.py (bf16, fp8) and PMC of the flagship pt4 vs
# hipBLASLt (bf16, MX-fp8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_36
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for dt in bfloat16 float8_e4m3fn; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$dt -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --dtype $dt > $R/$O/prof_bench_$dt.json 2> $R/$O/prof_bench_$dt.err || { tail -20 $R/$O/prof_bench_$dt.err; exit 1; }
  f=$(find /tmp/kt_$dt -name '*kernel_stats.csv' | head -1)
  cp "$f" $R/$O/kernel_stats_$dt.csv
  head -3 $R/$O/kernel_stats_$dt.csv | cut -c1-220
done
for dt in bfloat16 mx; do
  if [ $dt = mx ]; then A="--dtype float8_e4m3fn --mode mx"; else A="--dtype bfloat16"; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d /tmp/pmc_$dt -o p -- python3 $R/scripts/prof_gemm.py -m 65536 -n 1024 -k 1024 --tiles pt4 --hipblaslt --iters 5 $A > $R/$O/pmc_$dt.log 2>&1 || { tail $R/$O/pmc_$dt.log; exit 1; }
  python3 $R/scripts/pmc_summary.py $(find /tmp/pmc_$dt -name "*.db") > $R/$O/pmc_flagship_$dt.txt 2>&1
  grep -A10 "pt4_kernel\|hipBLASLt" $R/$O/pmc_flagship_$dt.txt | head -24
done
