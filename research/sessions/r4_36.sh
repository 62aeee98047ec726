# round 4 / 36: CU-split RCCL-fed fused candidate at world 1; native suite subset
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_36
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_native_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
TL="coll_pipeline/rccl/s4/fused,coll_pipeline/rccl/s4/fused/cumask"
for b in 32 6 64; do
  timeout -k 10 200 python -u scripts/plan_budget.py --world 8 --candidates "$TL" --rccl-blocks $b --iters 20 > $O/b$b.txt 2>&1; rc=$?
  echo "== blocks $b rc=$rc"; grep "fused" $O/b$b.txt | cut -c1-110
done
exit 0
