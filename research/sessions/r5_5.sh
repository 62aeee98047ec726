# round 5 / 5: in-launch K-split reduction (whole-tile ticket, sc1 hand-off, the other slice's
# partial added in place in two batches of 16 loads): tests, config #2 timing + kernel stats;
# gated-GEMM placement diagnostic; flagship C-store cache-policy A/B (DDLB_PT4_CAUX)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_native_gpu.py tests/test_gemm_gpu.py -k "ksplit or split_k" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
timeout -k 10 300 python -u scripts/bench_gemm.py --shapes 3 --tiles auto,pt4 --rounds 5 --check > $O/gemm_c2.txt 2>&1 || { echo "bench_gemm failed"; tail -20 $O/gemm_c2.txt; exit 1; }
grep -E "x|ms" $O/gemm_c2.txt | head -20
timeout -k 10 300 python bench.py -m 8192 -n 1024 -k 8192 --steps 50 --warmup 10 > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || { echo "bench failed"; tail -20 $O/bench_c2_bf16.err; exit 1; }
cut -c1-300 $O/bench_c2_bf16.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o c2 --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_gemm.py --shapes 3 --tiles auto --rounds 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
grep -h "pt4" $O/prof/*kernel_stats.csv | cut -c1-220
timeout -k 10 400 python -u scripts/diag_gate_placement.py --configs 32:32,32:64,32:256,24:8,24:32,24:256,16:16,16:64 > $O/gate_placement.txt 2>&1 || { echo "diag failed"; tail -20 $O/gate_placement.txt; exit 1; }
cat $O/gate_placement.txt
timeout -k 10 500 python -u scripts/ab_env_gemm.py --knob DDLB_PT4_CAUX --values 18,16,19,2 --shapes 0,6 --rounds 3 > $O/ab_caux_bf16.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab_caux_bf16.txt; exit 1; }
tail -12 $O/ab_caux_bf16.txt
