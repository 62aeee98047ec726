# t4 write-through C stores: numerics (GEMM + native suites), t4 A/B, smoke, bench N=1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2s4_20
mkdir -p $O
F="amdgpu.ids\|socket.cpp"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -a "FAILED\|Error" $O/gpu_tests.log | tail -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for v in wt nt wt nt; do
  if [ $v = nt ]; then export DDLB_PT4_NT_STORES=1; else unset DDLB_PT4_NT_STORES; fi
  timeout -k 10 300 python scripts/bench_gemm.py --rounds 3 --iters 20 --tiles auto,t4 --modes auto --shapes 0,2 > $O/gemm_$v.log 2>&1; rc=$?; echo "== C stores: $v"; grep -v "$F" $O/gemm_$v.log | grep "native\|bfloat16" | head -8; [ $rc -eq 0 ] || exit $rc
done
unset DDLB_PT4_NT_STORES
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
grep -a "\[bench\]" $O/bench.log; grep metric $O/bench.log | cut -c1-250
