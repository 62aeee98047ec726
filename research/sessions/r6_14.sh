# round 6 / 14: validation of the round-6 tree with the C park: whole GPU suite, smoke, bench N=1 (bf16 and fp8
# flagship, driver arguments), kernel-trace stats of both benches, PMC of the flagship pt4 vs
# hipBLASLt (bf16, MX-fp8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_14
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; grep -v "^  File\|^    " $O/gpu_tests.txt | tail -40; exit 1; }
tail -n 1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-400 $O/bench_bf16.json
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --dtype float8_e4m3fn > $O/bench_fp8.json 2> $O/bench_fp8.err || { echo "bench fp8 failed"; tail -20 $O/bench_fp8.err; exit 1; }
cut -c1-400 $O/bench_fp8.json
cd /tmp
for dt in bfloat16 float8_e4m3fn; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$dt -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --dtype $dt > $R/$O/prof_bench_$dt.json 2> $R/$O/prof_bench_$dt.err || { tail -20 $R/$O/prof_bench_$dt.err; exit 1; }
  f=$(find /tmp/kt_$dt -name '*kernel_stats.csv' | head -1)
  cp "$f" $R/$O/kernel_stats_$dt.csv
  head -5 $R/$O/kernel_stats_$dt.csv | cut -c1-220
done
for dt in bfloat16 mx; do
  if [ $dt = mx ]; then A="--dtype float8_e4m3fn --mode mx"; else A="--dtype bfloat16"; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d /tmp/pmc_$dt -o p -- python3 $R/scripts/prof_gemm.py -m 65536 -n 1024 -k 1024 --tiles pt4 --hipblaslt --iters 5 $A > $R/$O/pmc_$dt.log 2>&1 || { tail $R/$O/pmc_$dt.log; exit 1; }
  python3 $R/scripts/pmc_summary.py $(find /tmp/pmc_$dt -name "*.db") > $R/$O/pmc_flagship_$dt.txt 2>&1
  cat $R/$O/pmc_flagship_$dt.txt | head -40
done
