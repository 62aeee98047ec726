# round 6 / 37: in-tile staging (stage_dma, no tile-change test) in the gated pt4 branch -- the in-kernel
# all-gather GEMM at world 1 (scripts/bench_agk_world1.py: gated pt4 + copy workgroups, and the plain
# ungated GEMM beside it), the .so before / after alternated twice on one box; then the GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_37
mkdir -p $O
export TMPDIR=/tmp
SO=ddlb_amd/_C.cpython-310-x86_64-linux-gnu.so
for r in 1 2; do
  for v in before after; do
    cp research/abso/$v.so $SO
    echo "== $v (round $r)" >> $O/agk.txt
    timeout -k 10 200 python -u scripts/bench_agk_world1.py --ctas 32 --iters 100 >> $O/agk.txt 2>&1 || { echo "agk $v failed"; tail -20 $O/agk.txt; exit 1; }
  done
done
grep -v "^/opt" $O/agk.txt
cp research/abso/after.so $SO
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; grep -v "^  File\|^    " $O/gpu_tests.txt | tail -40; exit 1; }
tail -n 1 $O/gpu_tests.txt
