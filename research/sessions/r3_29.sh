# PMC of the VALU-free pt4 vs hipBLASLt: flagship 65536x1024x1024 and 8192^3 (MFMA busy, waits, LDS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_29
mkdir -p $O
cd /tmp
for shape in "65536 1024 1024" "8192 8192 8192"; do
  set -- $shape
  tag=${1}x${2}x${3}
  for set in "SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
    timeout -s KILL 120 rocprofv3 --pmc $set -d /tmp/pmc_$tag -o p -- python3 $GRAFT_REPO_ROOT/scripts/prof_gemm.py -m $1 -n $2 -k $3 --tiles pt4 --hipblaslt --iters 5 > $GRAFT_REPO_ROOT/$O/pmc_$tag.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/pmc_$tag.log; exit 1; }
    python3 $GRAFT_REPO_ROOT/scripts/pmc_summary.py $(find /tmp/pmc_$tag -name "*.db") --match "" 2>&1 | grep -A12 "pt4_kernel\|hipBLASLt 256\|Cijk" > $GRAFT_REPO_ROOT/$O/pmc_$tag.txt
    echo "== $tag"; cat $GRAFT_REPO_ROOT/$O/pmc_$tag.txt
  done
done
