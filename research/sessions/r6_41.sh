# round 6 / 41: PMC of the final pt4 vs hipBLASLt at 8192^3 and 16384x8192x8192 (bf16), one process each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_41
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for shp in "8192 8192 8192" "16384 8192 8192"; do
  set -- $shp
  tag=${1}x${2}x${3}
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d /tmp/pmc_$tag -o p -- python3 $R/scripts/prof_gemm.py -m $1 -n $2 -k $3 --tiles pt4 --hipblaslt --iters 5 --dtype bfloat16 > $R/$O/pmc_$tag.log 2>&1 || { tail $R/$O/pmc_$tag.log; exit 1; }
  python3 $R/scripts/pmc_summary.py $(find /tmp/pmc_$tag -name "*.db") > $R/$O/pmc_$tag.txt 2>&1
  grep -A10 "pt4_kernel\|hipBLASLt" $R/$O/pmc_$tag.txt | grep "==\|MFMA_BUSY\|GRBM\|duration"
done
