# round 4 / 4: PMC of the MX-fp8 pt4 vs hipBLASLt _scaled_mm (flagship and 8192^3), the r3_38
# counter set; then the harness-overhead breakdown under each HIP scheduling flag; smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4_4
mkdir -p $O
cd /tmp
for shape in "65536 1024 1024" "8192 8192 8192"; do
  set -- $shape
  tag=mx_${1}x${2}x${3}
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d /tmp/pmc_$tag -o p -- python3 $GRAFT_REPO_ROOT/scripts/prof_gemm.py -m $1 -n $2 -k $3 --tiles pt4 --dtype float8_e4m3fn --mode mx --hipblaslt --iters 5 > $GRAFT_REPO_ROOT/$O/pmc_$tag.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/pmc_$tag.log; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/pmc_summary.py $(find /tmp/pmc_$tag -name "*.db") --match "" > $GRAFT_REPO_ROOT/$O/pmc_$tag.txt 2>&1
  echo "== $tag"; grep -A11 "pt4_kernel\|Cijk\|hipBLASLt" $GRAFT_REPO_ROOT/$O/pmc_$tag.txt | head -60
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d /tmp/pmc2_$tag -o p -- python3 $GRAFT_REPO_ROOT/scripts/prof_gemm.py -m $1 -n $2 -k $3 --tiles pt4 --dtype float8_e4m3fn --mode mx --hipblaslt --iters 5 > $GRAFT_REPO_ROOT/$O/pmc2_$tag.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/pmc2_$tag.log; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/pmc_summary.py $(find /tmp/pmc2_$tag -name "*.db") --match "" > $GRAFT_REPO_ROOT/$O/pmc2_$tag.txt 2>&1
  echo "== $tag (2)"; grep -A9 "pt4_kernel\|Cijk\|hipBLASLt" $GRAFT_REPO_ROOT/$O/pmc2_$tag.txt | head -40
done
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/diag_harness_overhead.py > $O/harness.txt 2>&1 || { echo "harness diag failed"; tail -20 $O/harness.txt; exit 1; }
cat $O/harness.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 3 $O/smoke.txt
