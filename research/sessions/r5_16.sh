# round 5 / 16: PMC of the long-K GEMM (65536x1024x8192 bf16: -5 % vs hipBLASLt) -- LDS bank
# conflicts / LDS-array cycles / waits, and L2 hit rate, own pt4 vs hipBLASLt F.linear
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_16
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d /tmp/pmc_a -o p -- python3 $R/scripts/prof_gemm.py -m 65536 -n 1024 -k 8192 --tiles pt4 --hipblaslt --iters 3 > $R/$O/pmc_a.log 2>&1 || { tail $R/$O/pmc_a.log; exit 1; }
python3 $R/scripts/pmc_summary.py $(find /tmp/pmc_a -name "*.db") --match "" > $R/$O/pmc_longk_lds.txt 2>&1
grep -A11 "pt4\|hipBLASLt\|Cijk" $R/$O/pmc_longk_lds.txt | head -30
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum -d /tmp/pmc_b -o p -- python3 $R/scripts/prof_gemm.py -m 65536 -n 1024 -k 8192 --tiles pt4 --hipblaslt --iters 3 > $R/$O/pmc_b.log 2>&1 || { tail $R/$O/pmc_b.log; exit 1; }
python3 $R/scripts/pmc_summary.py $(find /tmp/pmc_b -name "*.db") --match "" > $R/$O/pmc_longk_inst_l2.txt 2>&1
grep -A10 "pt4\|hipBLASLt\|Cijk" $R/$O/pmc_longk_inst_l2.txt | head -30
