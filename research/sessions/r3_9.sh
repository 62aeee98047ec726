# Long-K GEMM: tile-raster group size A/B (DDLB_RASTER_G) and L2 behaviour (TCC PMC) of pt4 vs
# hipBLASLt at 8192^3 and 16384x8192x8192
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_9
mkdir -p $O
for g in 8 4 16 2; do
  DDLB_RASTER_G=$g timeout -k 10 200 python -u scripts/bench_gemm.py --tiles pt4 --shapes 5,6 --rounds 3 > $O/raster_g$g.log 2>&1 || { tail $O/raster_g$g.log; exit 1; }
  echo "G=$g"; grep -a "native\|hipblaslt_linear" $O/raster_g$g.log
done
cd /tmp
for set in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  n=$(echo $set | cut -c1-3)
  timeout -s KILL 120 rocprofv3 --pmc $set -d /tmp/pmc_$n -o p -- python3 $GRAFT_REPO_ROOT/scripts/prof_gemm.py -m 8192 -n 8192 -k 8192 --tiles pt4 --hipblaslt --iters 5 > $GRAFT_REPO_ROOT/$O/pmc_$n.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/pmc_$n.log; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/pmc_summary.py $(find /tmp/pmc_$n -name "*.db") --match "" 2>&1 | grep -A12 "pt4_kernel\|hipBLASLt 256" > $GRAFT_REPO_ROOT/$O/pmc_$n.txt
  cat $GRAFT_REPO_ROOT/$O/pmc_$n.txt
done
