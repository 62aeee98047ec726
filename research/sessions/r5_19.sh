# round 5 / 19: in-launch K-split with the canonical agent release / acquire hand-off (plain
# partial stores and loads): stale-partial rate with counters in uncached and cached memory, the
# in-launch / split tests, then the whole GPU suite, smoke, bench N=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_19
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/diag_ksr_memtype.py --runs 60 --fill nan > $O/diag_ksr_memtype_nan.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag_ksr_memtype_nan.txt; exit 1; }
grep "^{" $O/diag_ksr_memtype_nan.txt
timeout -k 10 300 python -u scripts/diag_ksr_memtype.py --runs 60 --fill zero -S 4 -m 4096 > $O/diag_ksr_memtype_zero_s4.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag_ksr_memtype_zero_s4.txt; exit 1; }
grep "^{" $O/diag_ksr_memtype_zero_s4.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_gpu.py -k "ksplit or split_k" > $O/ks_tests.txt 2>&1 || { echo "ks tests failed"; tail -30 $O/ks_tests.txt; exit 1; }
tail -n 1 $O/ks_tests.txt
timeout -k 10 300 python -u scripts/ab_ksplit_forms.py --tiles pt4 --checks 10 --splits 2 --shapes 8192x1024x8192,4096x1024x8192 > $O/ksplit_forms_bf16.txt 2>&1 || { echo "forms failed"; tail -30 $O/ksplit_forms_bf16.txt; exit 1; }
grep -v "^  check.* ok$" $O/ksplit_forms_bf16.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -n 1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bench failed"; tail -20 $O/bench_bf16.err; exit 1; }
cut -c1-300 $O/bench_bf16.json
timeout -k 10 400 python bench.py -m 8192 -n 1024 -k 8192 > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || { echo "bench c2 failed"; tail -20 $O/bench_c2_bf16.err; exit 1; }
cut -c1-300 $O/bench_c2_bf16.json
