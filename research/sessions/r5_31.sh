# round 5 / 31: PMC of the flagship GEMM, DEFER (default) vs the ONE schedule (DDLB_PT4_ONE=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_31
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp
for v in defer one; do
  if [ $v = one ]; then export DDLB_PT4_ONE=1; else unset DDLB_PT4_ONE; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d /tmp/pmc_$v -o p -- python3 $R/scripts/prof_gemm.py -m 65536 -n 1024 -k 1024 --tiles pt4 --iters 5 > $R/$O/pmc_$v.log 2>&1 || { tail $R/$O/pmc_$v.log; exit 1; }
  python3 $R/scripts/pmc_summary.py $(find /tmp/pmc_$v -name "*.db") --match "pt4" > $R/$O/pmc_flagship_$v.txt 2>&1
  cat $R/$O/pmc_flagship_$v.txt
done
