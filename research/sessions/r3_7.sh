# N=1 bench for fp8 (config #5 dtype) and tp_rowwise (config #3 shape) on own kernels only; the
# runner's --pmc option end to end; cs2 graph crash with faulthandler + native handler
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3_7
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dtype float8_e4m3fn > $O/bench_fp8.log 2>&1 || { tail -20 $O/bench_fp8.log; exit 1; }
grep -a "\[bench" $O/bench_fp8.log; grep -a metric $O/bench_fp8.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --primitive tp_rowwise -m 16384 -n 8192 -k 8192 > $O/bench_row.log 2>&1 || { tail -20 $O/bench_row.log; exit 1; }
grep -a "\[bench" $O/bench_row.log; grep -a metric $O/bench_row.log | cut -c1-300
timeout -k 10 300 python -m ddlb_amd --primitive tp_columnwise -m 65536 -n 1024 -k 1024 --dtype bfloat16 --impl "native" --impl "compute_only;size=unsharded;gemm=torch_nt" --num-iterations 20 --num-warmups 3 --pmc default --pmc-dir $O/pmc --output-csv $O/cli_pmc.csv > $O/cli_pmc.log 2>&1 || { tail -30 $O/cli_pmc.log; exit 1; }
tail -8 $O/cli_pmc.log | cut -c1-300
CFG='[["col/coll_pipeline/memcpy/cs2/graph", "col", {"algorithm": "coll_pipeline", "backend": "ipc", "s": 2, "copy_streams": 2, "graph": true}]]'
PORT=29667
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
  DDLB_PG_BACKEND=gloo DDLB_ALLOW_SHARED_GPU=1 DDLB_TEST_PROGRESS=1 DDLB_CRASH_BT=1 DDLB_GRAPH_CS2=1 \
  DDLB_TEST_CFGS="$CFG" timeout -k 10 100 python -u -X faulthandler tests/_ipc_worker.py > $O/cs2_graph_rank$r.log 2>&1 &
done
wait
tail -40 $O/cs2_graph_rank0.log
